"""Random stream spec v3 (include/rt_rng.h), CPU.

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
    with open(os.path.join(GOLDEN, "rng_v3.json")) as f:
        vecs = json.load(f)["vectors"]
    for v in vecs:
        vals, raw = oracle.rng_draws(v["seed"], v["pixel"], v["sample"], len(v["raw"]))
        assert raw.tolist() == v["raw"]
        assert [float.fromhex(h) for h in v["draws"]] == vals.tolist()


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
