"""Host sanitizer runs of the native IO library (SURVEY §5.2 race detection / sanitizers).

GPU AddressSanitizer / XNACK builds are not available on the MI355X pool, so the sanitizers run
on the host code: hfm_io.cpp + csrc/io/io_selftest.cpp under ASan+UBSan and under TSan (the
threaded loader).  The UBSan run found an out-of-range pointer computation in the Example
decoder's length checks (fixed with the length-based ``fits`` guard)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRCS = [os.path.join(ROOT, "csrc", "io", "hfm_io.cpp"), os.path.join(ROOT, "csrc", "io", "io_selftest.cpp")]


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_io_library_under_sanitizer(tmp_path, san):
    exe = str(tmp_path / "io_selftest")
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-msse4.2", f"-fsanitize={san}", "-fno-omit-frame-pointer",
           *SRCS, "-o", exe, "-lpthread"]
    if "undefined" in san:
        cmd.insert(5, "-fno-sanitize-recover=undefined")
    subprocess.run(cmd, check=True, capture_output=True, timeout=240)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0 and "io_selftest ok" in r.stdout, r.stdout + r.stderr
