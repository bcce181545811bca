"""Host-side sanitizer run of the kernel library: the pure-host entry points (GEMM argument
validation, record sizes the Python packers rely on) built with AddressSanitizer on the host half
(``-Xarch_host -fsanitize=address``) and executed on the CPU -- GPU ASan is not available on this pool."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc")
def test_host_checks_under_asan(tmp_path):
    exe = str(tmp_path / "host_checks")
    # gemm_glds.hip dispatches its 256 x 256 tiles to gemm_8ph.hip / gemm_4w.hip: link them too
    src = [os.path.join(ROOT, "tests", "native", "host_checks.cpp")] + [
        os.path.join(ROOT, "csrc", f) for f in ("gemm_glds.hip", "gemm_8ph.hip", "gemm_4w.hip", "kernels.hip",
                                                "splice.hip")]
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "csrc"),
           "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer", "-o", exe] + src
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1")
    run = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert run.returncode == 0, (run.stdout + run.stderr)[-4000:]
    assert "host checks passed" in run.stdout
