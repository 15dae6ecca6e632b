"""CPU: AddressSanitizer + UndefinedBehaviorSanitizer (and ThreadSanitizer) over the host code that
parses attacker-shaped bytes: the frag ->
descriptor parse, the tcache, the sync and async verify stages (host parse),
the precompile record walk, the gossip packet walks (CRDS values included), the shred walk and the
offload shared-memory link.

1. tests/csrc/sanitize_host.cpp: those product sources compiled with
   -fsanitize=address,undefined and driven with random / corrupted frags,
   instruction data and a hostile link peer (header words rewritten between
   calls).  Any sanitizer report aborts it.
2. The CPU test suites that exercise the same code run against ASan + UBSan
   builds of the product's host libraries (tests/csrc/Makefile asan; libasan
   preloaded into the test interpreter)."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(REPO, "tests", "_build")


def _lib(name):
    return subprocess.check_output(["gcc", "-print-file-name=" + name], text=True).strip()


def test_sanitized_driver():
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "tests", "csrc"), "sanitize"])
    r = subprocess.run([os.path.join(BUILD, "sanitize_host")], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
                                UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "sanitize_host: ok" in r.stdout
    # the random inputs reached every parser (counts printed by the driver)
    import re
    nums = [int(x) for x in re.findall(r"(\d+) (?:parsed ok|failed|bad|descriptors|published|taken|joins refused)",
                                        r.stdout)]
    assert len(nums) == 11 and min(nums) > 0, r.stdout
    m = re.search(r"device-parse stage (\d+) batches, (\d+) kicks", r.stdout)
    assert m and int(m.group(1)) > 0 and int(m.group(2)) > 0, r.stdout


def test_thread_sanitized_driver():
    """The same driver under ThreadSanitizer: the async stage's three threads
    (caller, poller, replayer) on the host-parse and the device-parse paths,
    the stand-in device queue answering PENDING and taking drain kicks."""
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "tests", "csrc"), "tsan"])
    r = subprocess.run([os.path.join(BUILD, "tsan_host")], capture_output=True, text=True, timeout=900,
                       env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "sanitize_host: ok" in r.stdout and "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]


def test_cpu_suites_against_asan_libraries():
    if not os.path.exists(os.path.join(REPO, "firedancer_amd", "build", "prod", "fd_ed25519_gpu_hsaco.inc")):
        subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "firedancer_amd")])
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "tests", "csrc"), "asan"])
    gpu_lib = os.path.join(BUILD, "asan", "libfd_ed25519_gpu.so")
    off_lib = os.path.join(BUILD, "asan", "libfd_verify_offload.so")
    for so in (gpu_lib, off_lib):   # really instrumented
        syms = subprocess.check_output(["nm", "-D", so], text=True)
        assert "__asan_report" in syms and "__ubsan_handle" in syms, so
    env = dict(os.environ, LD_PRELOAD=_lib("libasan.so") + " " + _lib("libubsan.so"),
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               FD_ED25519_GPU_LIB=gpu_lib, FD_VERIFY_OFFLOAD_LIB=off_lib)
    suites = ["tests/test_offload.py", "tests/test_abi.py", "tests/test_verify_stage.py", "tests/test_precompile.py",
              "tests/test_gossip.py", "tests/test_shred.py"]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-m", "not gpu", "-p", "no:cacheprovider"] + suites,
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert " passed" in r.stdout
