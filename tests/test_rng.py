"""Random stream spec v4 (include/rt_rng.h; v3's per-sample stream plus the
soft-shadow streams of v4), CPU.

The reference draws from Go's global, unseedable math/rand
(internal/math/random.go:8-14), so a Go run's draw order depends on the
goroutine schedule and no draw-level golden exists.  The
build defines a counter-keyed stream instead; these tests pin it three ways:
committed known-answer vectors, an independent Python statement of the spec,
and the header compiled by gcc (the jump-ahead coefficients the kernel's
cooperative soft shadows rely on).
"""
import json
import os
import subprocess
import textwrap

import numpy as np
import pytest

import oracle
import rng_spec  # tests/rng_spec.py
from conftest import GOLDEN, ROOT


def test_oracle_stream_matches_committed_vectors():
    with open(os.path.join(GOLDEN, "rng_v4.json")) as f:
        vecs = json.load(f)["vectors"]
    for v in vecs:
        vals, raw = oracle.rng_draws(v["seed"], v["pixel"], v["sample"], len(v["raw"]))
        assert raw.tolist() == v["raw"]
        assert [float.fromhex(h) for h in v["draws"]] == vals.tolist()


def test_oracle_soft_streams_match_committed_vectors():
    """v4: calculateSmartShadow's 16 points of a (sample, bounce, light) come
    from a stream of their own; the oracle's points and tries equal the
    committed vectors of the Python statement."""
    with open(os.path.join(GOLDEN, "rng_v4.json")) as f:
        vecs = json.load(f)["soft_vectors"]
    for v in vecs:
        pts, tries = oracle.soft_points(v["seed"], v["pixel"], v["sample"], v["depth"], v["light"])
        assert tries == v["tries"]
        assert [[float.fromhex(h) for h in p] for p in v["points"]] == pts.tolist()
        assert v["raw"] == rng_spec.soft_draws(v["seed"], v["pixel"], v["sample"], v["depth"], v["light"], 12)


def test_soft_streams_are_distinct_per_bounce_and_light():
    a = rng_spec.soft_draws(3, 77, 5, 0, 0, 6)
    others = [rng_spec.soft_draws(3, 77, 5, 1, 0, 6), rng_spec.soft_draws(3, 77, 5, 0, 1, 6),
              rng_spec.soft_draws(3, 77, 6, 0, 0, 6), rng_spec.draws(3, 77, 5, 6)[0]]
    assert all(a != o for o in others)


@pytest.mark.parametrize("seed,pixel,sample", [(1, 0, 0), (7, 5, 3), (2**63 + 5, 12345, 64), (3, 2**32 - 1, 7)])
def test_oracle_stream_matches_python_spec(seed, pixel, sample):
    raw, vals = rng_spec.draws(seed, pixel, sample, 200)
    ovals, oraw = oracle.rng_draws(seed, pixel, sample, 200)
    assert oraw.tolist() == raw
    assert ovals.tolist() == vals


def test_draws_are_in_unit_interval_and_keyed():
    vals, _ = oracle.rng_draws(1, 10, 0, 5000)
    assert vals.min() >= 0.0 and vals.max() < 1.0
    assert abs(vals.mean() - 0.5) < 0.02
    # distinct (pixel, sample) keys give distinct streams
    a, _ = oracle.rng_draws(1, 10, 0, 8)
    b, _ = oracle.rng_draws(1, 10, 1, 8)
    c, _ = oracle.rng_draws(1, 11, 0, 8)
    d, _ = oracle.rng_draws(2, 10, 0, 8)
    assert len({a.tobytes(), b.tobytes(), c.tobytes(), d.tobytes()}) == 4


def test_jump_ahead_identity():
    x = rng_spec.init(1, 99, 5)
    for j in (0, 1, 2, 3, 17, 64, 191, 192):
        a, c = rng_spec.jump(j)
        y = x
        for _ in range(j):
            y = rng_spec.step(y)
        assert (a * x + c) & rng_spec.M64 == y


def test_header_jump_coeffs_compiled_with_gcc(tmp_path):
    src = tmp_path / "j.c"
    src.write_text(textwrap.dedent("""
        #include <stdio.h>
        #include <inttypes.h>
        #include "rt_rng.h"
        int main(void) {
          const unsigned js[] = {0, 1, 2, 3, 17, 64, 191, 192};
          for (unsigned i = 0; i < sizeof js / sizeof js[0]; ++i) {
            uint64_t a, c;
            rt_pcg_jump_coeffs(js[i], &a, &c);
            printf("%u %" PRIu64 " %" PRIu64 "\\n", js[i], a, c);
          }
          rt_rng r;
          rt_rng_init(&r, rt_rng_seed_key(9), 4242, 17);
          for (int i = 0; i < 4; ++i) printf("d %a\\n", rt_rng_draw(&r));
          printf("s %" PRIu64 "\\n", rt_soft_state(rt_soft_key(rt_rng_seed_key(9), 4242, 17), 3, 1));
          return 0;
        }
    """))
    exe = tmp_path / "j"
    subprocess.run(["gcc", "-O2", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    lines = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    ds = []
    for ln in lines:
        if not ln:
            continue
        if ln.startswith("d "):
            ds.append(float.fromhex(ln[2:]))
            continue
        if ln.startswith("s "):
            assert int(ln[2:]) == rng_spec.soft_init(9, 4242, 17, 3, 1)
            continue
        j, a, c = (int(t) for t in ln.split())
        assert (a, c) == rng_spec.jump(j)
    assert ds == rng_spec.draws(9, 4242, 17, 4)[1]


def test_rejection_sampling_consumes_three_draws_per_try():
    # RandomVec3InUnitSphere (vector.go:132-139): the oracle's Lambertian
    # scatter consumes exactly 3 x tries draws of the stream
    import rtgo

    m = rtgo.Material()
    m.kind = rtgo.MATERIAL_KINDS["lambertian"]
    for sample in range(20):
        _, _, _, draws = oracle.scatter(m, (0, 0, 0), (0, 0, -1), (1, 0, 0, 0, 0, 0, 1, 1), 3, 8, sample)
        vals = np.array(rng_spec.draws(3, 8, sample, 300)[1])
        p = vals[: (len(vals) // 3) * 3].reshape(-1, 3) * 2 - 1
        first = int(np.argmax((p * p).sum(1) < 1))
        assert draws == 3 * (first + 1)
