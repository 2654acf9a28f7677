"""Build hygiene: the native build is keyed by source *content* (sha256 sidecars),
not mtimes -- an edit that keeps the old mtime still recompiles, an untouched tree
does not (ops/build.py)."""
import os
import shutil

import pytest

from apex_amd.ops import build


def _tiny_tree(tmp_path, monkeypatch):
    csrc = tmp_path / "csrc"
    csrc.mkdir()
    (csrc / "k.hip").write_text(
        "#include <hip/hip_runtime.h>\n"
        "__global__ void k(float* p) { p[threadIdx.x] = 1.0f; }\n")
    monkeypatch.setattr(build, "CSRC", csrc)
    monkeypatch.setattr(build, "BUILD", tmp_path / "_build")
    monkeypatch.setattr(build, "HIP_SOURCES", ["k.hip"])
    target = tmp_path / "libtiny.so"
    monkeypatch.setattr(build, "hip_target", lambda: target)
    return csrc / "k.hip", target


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="no hipcc")
def test_kernel_content_edit_rebuilds_even_with_old_mtime(tmp_path, monkeypatch):
    src, target = _tiny_tree(tmp_path, monkeypatch)
    build.build_hip()
    h1 = build.build_hash(target)
    assert h1 and target.exists()
    obj = tmp_path / "_build" / "k.hip.o"
    m_obj = obj.stat().st_mtime_ns

    # untouched tree: nothing recompiles, the hash is unchanged
    build.build_hip()
    assert obj.stat().st_mtime_ns == m_obj and build.build_hash(target) == h1

    # edit the kernel's content but put the mtime back to before the object was built
    st = src.stat()
    src.write_text(src.read_text().replace("1.0f", "2.0f"))
    os.utime(src, ns=(st.st_atime_ns, st.st_mtime_ns - 10**12))
    build.build_hip()
    h2 = build.build_hash(target)
    assert h2 != h1
    assert obj.stat().st_mtime_ns != m_obj  # the object was recompiled


def test_live_extension_has_a_hash_sidecar():
    """The in-tree library the GPU tests load carries the hash of the sources it was
    built from (``smoke()`` prints it); a rebuild check from the current sources agrees."""
    target = build.hip_target()
    if not target.exists():
        pytest.skip("extension not built")
    build.build_hip()  # no-op when current; rebuilds (and re-stamps) when sources moved on
    assert build.build_hash(target) is not None
