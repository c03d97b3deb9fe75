"""ASan/UBSan on the CPU build: the oracle's C restatement and the
product library's host-side translation units (pcdio.hip wire formats, pca.hip's
PCA::write / rotateFeature90 maps; host side only, no device code), driven over the
reference's own PCD clouds and PCA files.  A sanitizer report aborts the driver."""
import os
import shutil
import subprocess

import pytest

from conftest import GOLDEN, ROOT

SAN = ROOT / "tests" / "sanitize"
FIX = GOLDEN / "ref_fixtures"


@pytest.fixture(scope="module")
def built():
    if shutil.which("gcc") is None or not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("no toolchain")
    subprocess.run(["make", "-s", "-C", str(SAN), "-j4"], check=True, capture_output=True, text=True)
    return SAN / "build"


def _run(cmd):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return r.stdout


def test_oracle_under_asan_ubsan(built):
    pca = sorted(str(p) for p in (FIX / "models_offline_r").rglob("*") if p.is_file())
    assert "oracle_check ok" in _run([str(built / "oracle_check")] + pca)


def test_product_host_code_under_asan_ubsan(built, tmp_path):
    files = sorted(str(p) for p in (FIX / "pcd").glob("*.pcd"))
    files += sorted(str(p) for p in (FIX / "models_offline_r").rglob("*") if p.is_file())
    assert "host_check ok" in _run([str(built / "host_check"), str(tmp_path)] + files)
