"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer and under
ThreadSanitizer (GPU sanitizers are not available on this
pool, so only host code is instrumented): librtgo's loader, flattening, BVH
builder, schedule inputs, tile partitions, image writers and the
multi-threaded CPU oracle (its pthread tile queue mirrors the goroutines of
renderer.go:67-148), driven with every committed scene, the 10k-sphere scene
and malformed JSON (tests/c/sanitize_driver.cpp, tests/c/Makefile)."""
import importlib.util
import os
import subprocess

import pytest

from conftest import ROOT, SCENES

CDIR = os.path.join(ROOT, "tests", "c")


@pytest.fixture(scope="module")
def inputs(tmp_path_factory):
    subprocess.run(["make", "-C", CDIR, "-j4"], check=True, capture_output=True, timeout=900)
    spec = importlib.util.spec_from_file_location("gen_spheres", os.path.join(SCENES, "gen_spheres.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    tmp = tmp_path_factory.mktemp("san")
    big = tmp / "spheres10k.json"
    big.write_text(g.dumps(g.generate(10000)))
    return big, tmp


def _run(exe, inputs, env_extra):
    big, tmp = inputs
    # (verify_asan_link_order=0: the environment may preload a library ahead of the runtime)
    env = dict(os.environ, **env_extra)
    return subprocess.run([os.path.join(CDIR, "build", exe), SCENES, str(big), str(tmp)],
                          capture_output=True, text=True, timeout=900, env=env)


def test_host_code_is_clean_under_asan_and_ubsan(inputs):
    p = _run("sanitize_driver", inputs, {
        "ASAN_OPTIONS": "detect_leaks=1:halt_on_error=1:abort_on_error=0:verify_asan_link_order=0",
        "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"})
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-5000:]
    assert "sanitize_driver: 0 failures" in p.stdout
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr


def test_host_code_is_clean_under_tsan(inputs):
    p = _run("tsan_driver", inputs, {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"})
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-5000:]
    assert "sanitize_driver: 0 failures" in p.stdout
    assert "ThreadSanitizer" not in p.stderr
