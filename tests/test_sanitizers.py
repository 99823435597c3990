"""Host sanitizers ("Race detection / sanitizers"): the CPU
oracle (oracle/rv_oracle.c) and the host build of the product's traversal header
(tests/host/rv_host_trace.cpp instantiates include/rvgrt/rv_device.h) under AddressSanitizer +
UndefinedBehaviorSanitizer, every UB report fatal, running the CPU suites that exercise them:
world build (noise, CSDF, GI init / update), traversal KATs and random rays for every traversal
variant, whole golden frames and the second restatement's frames.  One pytest subprocess with
clang's shared ASan runtime preloaded (the sanitized libraries are dlopen'ed by ctypes)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/llvm/bin/clang"
SUITES = ["tests/test_oracle.py", "tests/test_host_trace.py", "tests/test_golden.py", "tests/test_trace_kat.py",
          "tests/test_np_shade.py"]


def _asan_runtime():
    p = subprocess.run([CLANG, "-print-file-name=libclang_rt.asan-x86_64.so"], capture_output=True, text=True)
    path = p.stdout.strip()
    if p.returncode != 0 or not os.path.isabs(path) or not os.path.exists(path):
        pytest.skip("clang's shared ASan runtime not found")
    return path


@pytest.mark.timeout(1500)
def test_oracle_and_host_traversal_under_asan_ubsan():
    rt = _asan_runtime()
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "san"], check=True)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "host"), "san"], check=True)
    env = dict(os.environ, RVGRT_SANITIZE="1", LD_PRELOAD=rt,
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0:exitcode=77",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1:exitcode=78", OMP_NUM_THREADS="4")
    chk = subprocess.run([sys.executable, "-c", "from oracle import oracle as O; print(O.lib()._name); "
                          "print(sum('asan' in l for l in open('/proc/self/maps')))"], cwd=ROOT, env=env,
                         capture_output=True, text=True, timeout=120)
    name, nmaps = chk.stdout.split()[-2:]
    assert name.endswith("liboracle_san.so") and int(nmaps) > 0, chk.stdout + chk.stderr   # the sanitized build ran
    p = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-m", "not gpu"]
                       + SUITES, cwd=ROOT, env=env, capture_output=True, text=True, timeout=1400)
    out = p.stdout + p.stderr
    assert "runtime error:" not in out, out[-4000:]            # UBSan
    assert "ERROR: AddressSanitizer" not in out, out[-4000:]
    assert p.returncode == 0, out[-4000:]
    assert " passed" in p.stdout
