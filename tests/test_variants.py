"""The image-changing timing experiments live only as patches
(scripts/variants/*.patch, applied by scripts/build_variant.sh to a scratch
copy): the product sources name none of their switches, and every patch
still applies to the current sources (CPU only; nothing is compiled)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

VARIANTS = os.path.join(ROOT, "scripts", "variants")
PATCHES = sorted(f for f in os.listdir(VARIANTS) if f.endswith(".patch"))


def test_product_sources_carry_no_experiment_switch():
    csrc = os.path.join(ROOT, "concurrent-raytracer-go_amd", "csrc")
    for name in os.listdir(csrc):
        with open(os.path.join(csrc, name), errors="replace") as f:
            assert "RT_EXP_" not in f.read(), name


@pytest.mark.skipif(shutil.which("patch") is None, reason="no patch(1)")
@pytest.mark.parametrize("name", PATCHES)
def test_patch_applies_to_the_current_sources(name, tmp_path):
    for d in ("include", os.path.join("concurrent-raytracer-go_amd", "csrc")):
        shutil.copytree(os.path.join(ROOT, d), tmp_path / d)
    with open(os.path.join(VARIANTS, name)) as f:
        p = subprocess.run(["patch", "-p1", "--dry-run", "-s"], stdin=f, cwd=tmp_path, capture_output=True, text=True)
    assert p.returncode == 0, p.stdout + p.stderr
