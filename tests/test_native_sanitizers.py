"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (sanitizers on host code only — GPU
ASan is not available on this pool).

* tests/native/test_validate.cpp — ad_merge_host's reply validation (cassandra-accord_amd/csrc/validate.h, the
  exact code the engine links) on canonical and fuzzed malformed replies;
* tests/native/oracle_asan.cpp — the CPU oracle (oracle/oracle.cpp) over seeded batches of every shape, all entry
  points (deps, merge incl. the fast-path mask, levels, MaxConflicts with a carried map, fetches).
A sanitizer report aborts the binary (-fno-sanitize-recover=all), failing the test."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
FLAGS = ["-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
         "-fno-sanitize-recover=all", "-Wno-subobject-linkage"]

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")


def _build_run(src, tmp_path, extra=()):
    exe = str(tmp_path / os.path.basename(src).replace(".cpp", ""))
    subprocess.check_call(["g++"] + FLAGS + [os.path.join(HERE, "native", src), "-o", exe] + list(extra))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    out = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "runtime error" not in out.stderr and "AddressSanitizer" not in out.stderr, out.stderr
    return out.stdout


def test_validate_under_sanitizers(tmp_path):
    assert "malformed rejected" in _build_run("test_validate.cpp", tmp_path)


def test_oracle_under_sanitizers(tmp_path):
    assert "oracle under ASan/UBSan" in _build_run("oracle_asan.cpp", tmp_path, ["-lpthread"])
