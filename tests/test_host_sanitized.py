"""AddressSanitizer + UndefinedBehaviorSanitizer on the CPU:

* the runtime's host-only code (pixiu_amd/csrc/px_host.h: CritBit index, key maps, block
  heap, worker pool) through tests/cpp/host_test.cpp, built with -fsanitize;
* the CPU restatement (oracle/pxo.cpp, `make -C oracle asan`) loaded into a python with
  libasan preloaded, running the golden-vector tests (KATs, README transcript, CRUD
  script, config corpora; the rotation corpora and the reinsert scenarios take ~10
  minutes under the sanitizers and run in tools/sanitize.sh)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gcc_lib(name):
    return subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_host_code_sanitized(tmp_path):
    exe = str(tmp_path / "host_test")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-fno-omit-frame-pointer", "-I", os.path.join(ROOT, "pixiu_amd", "csrc"),
                    os.path.join(ROOT, "tests", "cpp", "host_test.cpp"), "-o", exe, "-lpthread"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, ASAN_OPTIONS="halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host_test: ok" in r.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_oracle_sanitized():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)
    asan, ubsan = _gcc_lib("libasan.so"), _gcc_lib("libubsan.so")
    if not (os.path.exists(asan) and os.path.exists(ubsan)):
        pytest.skip("no sanitizer runtimes")
    env = dict(os.environ, LD_PRELOAD=f"{asan}:{ubsan}", ASAN_OPTIONS="detect_leaks=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               PXO_LIB=os.path.join(ROOT, "oracle", "_build", "libpxo_asan.so"))
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_oracle_golden.py"), "-k", "not rotation"],
                       capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert " passed" in r.stdout
