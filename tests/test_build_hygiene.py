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


def bench_profile_paths():
    """The PMC summaries bench.py reads by default (its --valu and --traffic defaults)."""
    import re

    with open(os.path.join(ROOT, "bench.py")) as f:
        src = f.read()
    paths = {}
    for opt in ("valu", "traffic"):
        m = re.search(rf'"--{opt}", default=os.path.join\(ROOT, "profiles", "([^"]+)"\)', src)
        assert m, f"bench.py --{opt} default not found"
        paths[opt] = os.path.join(ROOT, "profiles", m.group(1))
    return paths


def test_committed_profiles_name_one_build():
    """bench.py derives roofline.frac / roofline.hbm only from PMC summaries measured on the
    library it loads (by hash): the VALU and traffic summaries it reads by default must exist, hold the
    headline workload (BASELINE configs[1]), and name one library for every workload they hold."""
    import json

    hashes = {}
    for opt, path in bench_profile_paths().items():
        with open(path) as f:
            rows = [json.loads(line) for line in f if line.strip()] if path.endswith(".jsonl") else [json.load(f)]
        assert any(r.get("workload") == "random_spheres:1920x1080x500" for r in rows), (path, "no headline entry")
        for r in rows:
            assert r.get("librtx_sha256_16"), (path, r.get("workload"))
            hashes.setdefault(r["librtx_sha256_16"], []).append((opt, r["workload"]))
    assert len(hashes) == 1, {h: v[:3] for h, v in hashes.items()}


def test_library_carries_no_build_date():
    """librtx.so's bytes depend on its sources only (rtx_build_info names no build date), so the PMC
    summaries bench.py ties to the library's hash (profiles/valu_r03.json) survive a rebuild."""
    import re

    import rtx

    info = rtx.load().rtx_build_info().decode()
    assert "ABI 9" in info
    assert not re.search(r"(Jan|Feb|Mar|Apr|May|Jun|Jul|Aug|Sep|Oct|Nov|Dec) +\d+ +\d{4}|\d\d:\d\d:\d\d", info), info
