"""ASan + UBSan over the product's C++ host layer (SURVEY §5 race /
sanitizer coverage; the reference runs `go test -race`, Makefile:24-27):
tm_host_abi.cpp, tm_light_abi.cpp, tm_types.h, tm_light.h, pool.cpp are
built with -fsanitize=address,undefined (tests/native/Makefile `asan`) into
the CPU harness, and the host-layer suites run against that build in a
child process with the sanitizer runtimes preloaded.  Any heap / stack
overflow, use-after-free or undefined behaviour aborts the child."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SUITES = ["tests/test_commit_verify.py", "tests/test_light_mbt.py", "tests/test_batch_verifier.py",
          "tests/test_failure_handling.py", "tests/test_chains.py", "tests/test_vote_set.py"]


def _runtime(name):
    return subprocess.run(["gcc", "-print-file-name=" + name], capture_output=True, text=True).stdout.strip()


def test_host_layer_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "tests", "native"), "asan"], check=True)
    so = os.path.join(REPO, "oracle", "_build", "asan", "libcommitcheck.so")
    pre = " ".join([_runtime("libasan.so"), _runtime("libubsan.so")] +
                   ([os.environ["LD_PRELOAD"]] if os.environ.get("LD_PRELOAD") else []))
    env = dict(os.environ, LD_PRELOAD=pre, TMV_COMMITCHECK_SO=so,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    out = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "not gpu", "-p", "no:cacheprovider"] +
                         SUITES, cwd=REPO, env=env, capture_output=True, text=True, timeout=1200)
    assert out.returncode == 0, (out.stdout[-3000:], out.stderr[-3000:])
    assert "ERROR: AddressSanitizer" not in out.stderr and "runtime error:" not in out.stderr
    assert " passed" in out.stdout
