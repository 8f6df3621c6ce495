"""Host-side native code under AddressSanitizer + UndefinedBehaviorSanitizer.

The checkpoint writer / readers in ``csrc/json_format.cpp`` parse files a user can hand the
service, so they are built here as a plain host program with ``-fsanitize=address,undefined``
(``tests/native/json_sanitize.cpp``) and driven three ways:

* ``roundtrip`` — random strided arrays (denormals, huge, integers, signed zeros, raw bit
  patterns) written by ``format_json_array`` and read back by ``scan_json_arrays`` bit-exactly;
* ``fuzz`` — 20,000 truncated / mutated checkpoints into ``scan_json_arrays`` and
  ``json_null_keys`` (exact-size heap buffers, so an over-read is an ASan report);
* ``repr`` — ``repr_double`` against Python's ``repr(float)`` on the same doubles.

GPU code is never sanitized on this pool (no GPU ASan / xnack); this covers the host parser.
"""
import math
import os
import random
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "penr_oz_neural_network_torch_amd", "csrc")


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    out = str(tmp_path_factory.mktemp("san") / "json_sanitize")
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
           "-fno-sanitize-recover=undefined", "-I", CSRC, os.path.join(ROOT, "tests", "native", "json_sanitize.cpp"),
           os.path.join(CSRC, "json_format.cpp"), "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0 and "sanitize" in r.stderr:
        pytest.skip("sanitizer runtime unavailable: " + r.stderr[-200:])
    assert r.returncode == 0, r.stderr
    return out


def _run(exe, mode, stdin=None):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, mode], input=stdin, capture_output=True, text=True, env=env, timeout=300)
    assert "ERROR: AddressSanitizer" not in r.stderr, r.stderr[-3000:]
    assert "runtime error:" not in r.stderr, r.stderr[-3000:]
    assert r.returncode == 0, (r.returncode, r.stdout[-500:], r.stderr[-3000:])
    return r.stdout


def test_roundtrip_bit_exact_under_sanitizers(harness):
    assert "roundtrip ok" in _run(harness, "roundtrip")


def test_malformed_checkpoints_are_rejected_cleanly(harness):
    out = _run(harness, "fuzz")
    parsed, rejected = (int(x) for x in out.split("parsed")[1].split("rejected"))
    assert rejected > 0 and parsed > 0


def test_repr_double_matches_python(harness):
    rng = random.Random(5)
    xs = [0.1, 5e-324, -0.0, 0.0, 1.7976931348623157e308, 1e16, 1e-7, 123456789.0, 2.0 ** 53, 1 / 3]
    xs += [rng.uniform(-1e6, 1e6) for _ in range(300)]
    xs += [math.ldexp(rng.random(), rng.randint(-1074, 1023)) for _ in range(300)]
    out = _run(harness, "repr", "\n".join(float.hex(x) for x in xs) + "\n").split()
    assert out == [repr(x) for x in xs]
