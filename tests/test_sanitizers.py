"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md
§5; GPU sanitizers are not available on this pool, so only host code is
instrumented): librtgo's loader, flattening, BVH builder, schedule inputs,
image writers and the multi-threaded CPU oracle, driven with every
committed scene, the 10k-sphere scene and malformed JSON
(tests/c/sanitize_driver.cpp, tests/c/Makefile)."""
import os
import subprocess

from conftest import ROOT, SCENES


def test_host_code_is_clean_under_asan_and_ubsan(tmp_path):
    cdir = os.path.join(ROOT, "tests", "c")
    subprocess.run(["make", "-C", cdir, "-j4"], check=True, capture_output=True, timeout=600)
    from scene_cases import spheres10k_scene  # noqa: F401  (the generator)
    import importlib.util

    spec = importlib.util.spec_from_file_location("gen_spheres", os.path.join(SCENES, "gen_spheres.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    big = tmp_path / "spheres10k.json"
    big.write_text(g.dumps(g.generate(10000)))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    p = subprocess.run([os.path.join(cdir, "build", "sanitize_driver"), SCENES, str(big), str(tmp_path)],
                       capture_output=True, text=True, timeout=600, env=env)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-5000:]
    assert "sanitize_driver: 0 failures" in p.stdout
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr
