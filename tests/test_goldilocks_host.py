"""goldilocks.hpp and xfe.hpp compiled for the host: the closed-form to_mont equals the Montgomery product by
2^128 mod p (BFieldElement::new -> raw word) on edge words (limbs near 0, 2^31, 2^32 - 1; words
around p and 2^64) and 2M random words.  CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_to_mont_closed_form_matches_montgomery_product(tmp_path):
    exe = tmp_path / "to_mont_check"
    subprocess.check_call([HIPCC, "-O2", "-std=c++17", "-x", "hip", "--offload-arch=gfx950",
                           "-I", os.path.join(ROOT, "neptune-core_amd", "csrc"),
                           os.path.join(ROOT, "tests", "native", "to_mont_check.cpp"), "-o", str(exe)],
                          stderr=subprocess.DEVNULL)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "bad 0" in out.stdout


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_mds_folded_round_constant_matches_stepwise(tmp_path):
    """mds_ark's folded reduction (round constant in the accumulators, one multiply-add with carry-out)
    equals twenty-first's reduce-then-add for every Tip5 round constant."""
    exe = tmp_path / "mds_fold_check"
    subprocess.check_call([HIPCC, "-O2", "-std=c++17", "-x", "hip", "--offload-arch=gfx950",
                           "-I", os.path.join(ROOT, "neptune-core_amd", "csrc"),
                           os.path.join(ROOT, "tests", "native", "mds_fold_check.cpp"), "-o", str(exe)],
                          stderr=subprocess.DEVNULL)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "bad 0" in out.stdout


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_lazy_xfe_product_and_field_sum_match_integer_arithmetic(tmp_path):
    """x_mul's lazily reduced form (nine 128-bit products, three Montgomery reductions) and gl_add's
    single-select form equal 128-bit integer arithmetic mod p on edge and 3M random operands."""
    exe = tmp_path / "xfe_check"
    subprocess.check_call([HIPCC, "-O2", "-std=c++17", "-x", "hip", "--offload-arch=gfx950",
                           "-I", os.path.join(ROOT, "neptune-core_amd", "csrc"),
                           os.path.join(ROOT, "tests", "native", "xfe_check.cpp"), "-o", str(exe)],
                          stderr=subprocess.DEVNULL)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "bad 0" in out.stdout


def test_staging_copy_streaming_stores_match_memcpy(tmp_path):
    """The staging copy's streaming-store word copy (host_copy.hpp) equals memcpy at every 8-byte
    destination / source alignment and lengths 0-300 and beyond, and writes nothing outside the
    destination (ASan + UBSan build)."""
    import shutil
    gxx = shutil.which("g++")
    if not gxx:
        pytest.skip("g++ not available")
    exe = tmp_path / "copy_check"
    subprocess.check_call([gxx, "-O2", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                           "-I", os.path.join(ROOT, "neptune-core_amd", "csrc"),
                           os.path.join(ROOT, "tests", "native", "copy_check.cpp"), "-o", str(exe)])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "bad 0" in out.stdout
