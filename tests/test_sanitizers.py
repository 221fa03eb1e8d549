"""Host runtime under AddressSanitizer+UBSan and ThreadSanitizer.

Builds the host-only library and tests/native/native_tests.cc with the CMake presets
(CMakePresets.json) and runs the driver: HostCache against an oracle, HTTP parser
splits + garbage, StreamBuf, ketama ejection, the host router (worker pool; hot table
swapped under concurrent readers), and the multi-threaded proxy (4 reactor
threads) over DRAM, fault-injected DRAM (timer thread) and a memcached-protocol node
(IO thread). Any sanitizer report fails the test."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("cmake") is None or shutil.which("ninja") is None,
                    reason="cmake/ninja not available")
@pytest.mark.parametrize("preset", ["asan", "tsan"])
def test_native_driver_under_sanitizer(preset):
    jobs = str(min(8, os.cpu_count() or 1))
    for cmd in (["cmake", "--preset", preset], ["cmake", "--build", "--preset", preset, "-j", jobs]):
        p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=900)
        assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=0"
    env["TSAN_OPTIONS"] = "halt_on_error=0:second_deadlock_stack=1"
    # (the presets build under /tmp/shellac-cmake: generated CMake sources stay out of the
    # source tree)
    exe = os.path.join("/tmp/shellac-cmake", preset, "shellac_native_tests")
    p = subprocess.run([exe], cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    report = p.stdout[-3000:] + p.stderr[-6000:]
    assert "ALL OK" in p.stdout, report
    assert "Sanitizer" not in p.stderr and "runtime error" not in p.stderr, report
    assert p.returncode == 0, report
