"""ASan/UBSan on the host code (SURVEY.md §5 "race detection / sanitizers"): the CPU oracle
(oracle/hdb_oracle.c) and the product's host C++ (csrc/flat.cpp, formats.cpp,
local_model.cpp) are rebuilt with -fsanitize=address,undefined by tests/sanitize/Makefile and
driven over tie-heavy seeded inputs, error paths and malformed records.  A sanitizer report
aborts the driver (non-zero exit).  The same host code is also built with -fsanitize=thread and
run from 8 threads at once (host_tsan: the C3/C5 local-model pool's host half), each thread's
result digest checked against a serial run of its seed.  GPU sanitizers are not available on the GPU pool; the
kernels are covered by the bit-exact parity tests instead."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def built(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("sanitize"))
    r = subprocess.run(["make", "-s", "-C", os.path.join(HERE, "sanitize"), f"OUT={out}"], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return out


@pytest.mark.parametrize("exe", ["oracle_asan", "host_asan"])
def test_host_code_under_asan_ubsan(built, exe):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(built, exe)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "asan ok" in r.stdout, r.stdout + r.stderr[-4000:]


def test_host_code_threaded_under_tsan(built):
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
    r = subprocess.run([os.path.join(built, "host_tsan"), "8", "16"], capture_output=True, text=True, timeout=600,
                       env=env)
    assert r.returncode == 0 and "host tsan ok" in r.stdout, r.stdout + r.stderr[-4000:]
