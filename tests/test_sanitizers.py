"""Host-side sanitizer builds (SURVEY §5 "race detection / sanitizers"), CPU only.

* oracle/_san/oracle_san — the CPU oracle (oracle/lqr_oracle.c) under AddressSanitizer +
  UBSan, driven over every entry point (oracle/san_main.c);
* lqr.jl_amd/csrc/build/api_san — the C ABI (lqrx_api.cpp: validation, KKT structure
  layout, generator, last-error buffer) with ASan + UBSan on the host side only
  (-Xarch_host; GPU sanitizers are not available on this pool), driven by api_san_main.cpp.
A sanitizer report aborts the program (-fno-sanitize-recover), failing the test.
"""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(make_dir, exe):
    jobs = str(min(8, os.cpu_count() or 1))
    subprocess.run(["make", "-s", "-j", jobs, "-C", os.path.join(ROOT, make_dir), "asan"], check=True, timeout=900)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(ROOT, exe)], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr
    return r.stdout


def test_oracle_under_asan_ubsan():
    assert "oracle sanitizer run: ok" in _run("oracle", "oracle/_san/oracle_san")


def test_abi_host_under_asan_ubsan(lqrx):
    assert "api sanitizer run: ok" in _run("lqr.jl_amd/csrc", "lqr.jl_amd/csrc/build/api_san")
