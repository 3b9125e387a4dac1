"""Build hygiene (CPU): a kernel source that does not compile fails `make`, even where the
Makefile filters hipcc's output through grep, and leaves no stale object behind."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("src", ["rtx_kernel", "rtx_ppm"])
def test_broken_source_fails_make(built, tmp_path, src):
    pkg = tmp_path / "raytracer-go_amd"
    shutil.copytree(os.path.join(ROOT, "raytracer-go_amd", "csrc"), pkg / "csrc")
    shutil.copy(os.path.join(ROOT, "raytracer-go_amd", "Makefile"), pkg / "Makefile")
    shutil.copytree(os.path.join(ROOT, "include"), tmp_path / "include")
    # a stale object from an earlier good build must not survive the failed one
    (pkg / "build").mkdir()
    stale = pkg / "build" / f"{src}.o"
    shutil.copy(os.path.join(ROOT, "raytracer-go_amd", "build", f"{src}.o"), stale)
    path = pkg / "csrc" / f"{src}.hip"
    path.write_text("#error deliberately broken source (tests/test_build_hygiene.py)\n" + path.read_text())
    os.utime(path, None)
    r = subprocess.run(["make", "-C", str(pkg), f"build/{src}.o"], capture_output=True, text=True, timeout=600)
    assert r.returncode != 0, r.stdout + r.stderr
    assert "deliberately broken" in r.stdout + r.stderr
    assert not stale.exists()


def test_committed_profiles_name_one_build():
    """bench.py derives roofline.frac / roofline.hbm only from PMC summaries measured on the
    library it loads (by hash): the committed VALU and traffic summaries must name the same one."""
    import json

    hashes = set()
    for name in ("valu_r03.json", "traffic_r03.json"):
        with open(os.path.join(ROOT, "profiles", name)) as f:
            d = json.load(f)
        assert d.get("librtx_sha256_16"), name
        assert d["workload"] == "random_spheres:1920x1080x500"
        hashes.add(d["librtx_sha256_16"])
    assert len(hashes) == 1, hashes


def test_library_carries_no_build_date():
    """librtx.so's bytes depend on its sources only (rtx_build_info names no build date), so the PMC
    summaries bench.py ties to the library's hash (profiles/valu_r03.json) survive a rebuild."""
    import re

    import rtx

    info = rtx.load().rtx_build_info().decode()
    assert "ABI 8" in info
    assert not re.search(r"(Jan|Feb|Mar|Apr|May|Jun|Jul|Aug|Sep|Oct|Nov|Dec) +\d+ +\d{4}|\d\d:\d\d:\d\d", info), info
