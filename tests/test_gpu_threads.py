"""The C3/C5 model pool's concurrency, reduced to its library calls:
tools/thread_stress.py runs local models (bubble K5 cores, block and cooperative Prims, host
cluster tree + FOSC), leaf exact MSTs (K1t + K2b) and batched leaf Prims from 8 host threads,
one context and stream each, on 12 hardware queues, and checks every job's digest against a
serial pass.  It runs in its own process because HIP reads GPU_MAX_HW_QUEUES at start-up;
faulthandler and the library's native backtrace (HDB_NATIVE_BACKTRACE) put both stacks on
stderr if anything crashes."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_model_pool_threads_equal_serial():
    env = dict(os.environ, HDB_HW_QUEUES="12", HDB_NATIVE_BACKTRACE="1")
    r = subprocess.run([sys.executable, "-X", "faulthandler", os.path.join(ROOT, "tools", "thread_stress.py"),
                        "--threads", "8", "--rounds", "1", "--quick"], capture_output=True, text=True, timeout=240,
                       env=env, cwd=ROOT)
    assert r.returncode == 0 and "thread stress ok" in r.stdout, r.stdout[-3000:] + r.stderr[-6000:]
