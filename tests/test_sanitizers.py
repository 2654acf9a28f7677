"""Host C++ under AddressSanitizer + UndefinedBehaviorSanitizer.

The replay core (_apex_cpu: segment trees, PER batch ops, n-step returns) is rebuilt
with ``-fsanitize=address,undefined`` into a temp dir, and the host replay / n-step test
modules run against it in a child Python with libasan preloaded.  Any heap overflow,
use-after-free or UB (signed overflow, misaligned access, bad shift, ...) aborts the
child.  GPU code is not covered: GPU ASan / XNACK runs are not available on the pool.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.slow
def test_replay_core_under_asan_ubsan(tmp_path):
    from apex_amd.ops import build

    try:
        build.build_cpu(force=True, out_dir=tmp_path, sanitize=True)
    except Exception as e:  # toolchain without sanitizer runtimes
        pytest.skip(f"sanitizer build unavailable: {e}")
    env = build.sanitizer_env(tmp_path)
    if not os.path.exists(env["LD_PRELOAD"]):
        pytest.skip("libasan not found")
    # the child proves it loaded the sanitized module, then runs the host replay tests
    code = ("import sys; sys.path.insert(0, %r); from apex_amd import ops; m = ops.cpu(); "
            "assert m.__file__.startswith(%r), m.__file__; import pytest; "
            "sys.exit(pytest.main(['-q', '-x', '-p', 'no:cacheprovider', %r, %r]))"
            % (ROOT, str(tmp_path), os.path.join(ROOT, "tests", "test_replay_host.py"),
               os.path.join(ROOT, "tests", "test_nstep_host.py")))
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT, capture_output=True, text=True, timeout=900)
    out = r.stdout[-3000:] + r.stderr[-3000:]
    assert r.returncode == 0, out
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out
