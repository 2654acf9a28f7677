"""In-tree native build driver (no torch.utils.cpp_extension, no hipify).

Builds two pybind11 extension modules next to this file:

* ``_apex_cpu``  -- host C++17 (g++): segment trees / PER batch ops used by the
  reference-compatible replay buffers (reference memory.py:10-320).
* ``_apex_hip``  -- HIP C++ for gfx950 only (``hipcc --offload-arch=gfx950``): the
  HBM replay, n-step batcher, synthetic vector env, fused loss / optimizer and the
  MFMA conv/FC kernels of the Nature-CNN dueling network.

Neither module links libtorch: kernels take raw device pointers and the HIP stream
handle of the caller, so they are captured by ``torch.cuda.CUDAGraph`` like any
other work on that stream.  ``libamdhip64.so.7`` resolves to the copy torch has
already loaded (same SONAME), so ``import torch`` must precede the import of
``_apex_hip`` (``apex_amd.ops`` does that).

Usage: ``python -m apex_amd.ops.build [--force] [--jobs N] [--only cpu|hip]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
BUILD = HERE / "_build"
ARCH = "gfx950"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))

CPU_SOURCES = ["cpu_replay.cpp"]
HIP_SOURCES = [
    "hip_bindings.cpp",
    "replay_kernels.hip",
    "actor_kernels.hip",
    "learner_kernels.hip",
    "conv_kernels.hip",
    "conv_bwd_kernels.hip",
    "aql_kernels.hip",
    "aql_engine_kernels.hip",
    "conv1_kernels.hip",
    "fc_kernels.hip",
    "loss_heads_kernels.hip",
    "f32_kernels.hip",
    "ipc_kernels.hip",
    "comm.cpp",
    "ipc.cpp",
]


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _py_includes() -> list[str]:
    import pybind11

    return [f"-I{sysconfig.get_paths()['include']}", f"-I{pybind11.get_include()}", f"-I{CSRC}"]


def _headers() -> list[Path]:
    return sorted(CSRC.glob("*.h")) + sorted(CSRC.glob("*.cuh")) + sorted(CSRC.glob("*.hpp"))


def _digest(parts: list) -> str:
    """sha256 over the *contents* of the given files and the given strings (flags,
    compiler path).  mtimes are never trusted: a tree unpacked on another machine, a
    ``git checkout`` or a copy can leave an old binary newer than its edited source."""
    h = hashlib.sha256()
    for p in parts:
        if isinstance(p, Path):
            h.update(b"F" + p.name.encode() + b"\0")
            h.update(p.read_bytes() if p.exists() else b"<missing>")
        else:
            h.update(b"S" + str(p).encode() + b"\0")
    return h.hexdigest()


def _sidecar(target: Path) -> Path:
    return target.with_name(target.name + ".sha256")


def build_hash(target: Path) -> str | None:
    """The content hash recorded beside ``target`` by the build that produced it."""
    sc = _sidecar(Path(target))
    return sc.read_text().strip() if sc.exists() else None


def _stale(target: Path, digest: str) -> bool:
    return not target.exists() or build_hash(target) != digest


def _stamp(target: Path, digest: str) -> None:
    _sidecar(target).write_text(digest + "\n")


def _run(cmd: list[str]) -> None:
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + proc.stdout + proc.stderr)
        raise RuntimeError(f"native build failed: {cmd[-1] if cmd else ''}")
    if proc.stderr.strip() and os.environ.get("APEX_BUILD_VERBOSE"):
        sys.stderr.write(proc.stderr)


def cpu_target() -> Path:
    return HERE / f"_apex_cpu{_ext_suffix()}"


def hip_target() -> Path:
    return HERE / f"_apex_hip{_ext_suffix()}"


SANITIZE_FLAGS = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                  "-fno-sanitize-recover=undefined"]


def build_cpu(force: bool = False, out_dir: Path | None = None, sanitize: bool = False) -> Path:
    """``sanitize``: an ASan + UBSan build of the host replay core into
    ``out_dir`` -- load it with libasan preloaded (``sanitizer_env``)."""
    target = cpu_target() if out_dir is None else Path(out_dir) / cpu_target().name
    srcs = [CSRC / s for s in CPU_SOURCES]
    cxx = os.environ.get("CXX", "g++")
    opt = SANITIZE_FLAGS if sanitize else ["-O3"]
    cmd = [cxx, *opt, "-std=c++17", "-shared", "-fPIC", "-ffp-contract=off", "-fvisibility=hidden",
           *_py_includes(), *map(str, srcs), "-o", str(target)]
    digest = _digest([*srcs, *_headers(), *cmd[:-1]])
    if not force and not _stale(target, digest):
        return target
    _run(cmd)
    _stamp(target, digest)
    return target


def sanitizer_env(ext_dir: Path) -> dict:
    """Environment for a Python child that imports the sanitized ``_apex_cpu`` from
    ``ext_dir`` (``APEX_CPU_EXT_DIR``): libasan must be the first DSO loaded."""
    cxx = os.environ.get("CXX", "g++")
    asan = subprocess.run([cxx, "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    env = dict(os.environ)
    env.update(LD_PRELOAD=asan, APEX_CPU_EXT_DIR=str(ext_dir), APEX_NO_AUTOBUILD="1",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    return env


def _hipcc() -> str:
    cand = ROCM / "bin" / "hipcc"
    return str(cand) if cand.exists() else (shutil.which("hipcc") or "hipcc")


HIP_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-fvisibility=hidden",
    "-ffp-contract=fast-honor-pragmas",  # fast, except where a kernel pins its rounding (prio_mix)
    "-munsafe-fp-atomics",
    "-mcode-object-version=5",
    "-Wno-unused-result",
]


def build_hip(force: bool = False, jobs: int | None = None) -> Path:
    """Every object is keyed by the sha256 of its source, all headers and its full
    compile line (sidecar ``<obj>.sha256``); the library by the hashes of its objects and
    the link line.  ``build_hash(hip_target())`` identifies the binary that runs."""
    target = hip_target()
    BUILD.mkdir(exist_ok=True)
    srcs = [CSRC / s for s in HIP_SOURCES]
    hdrs = _headers()
    objs = []
    todo = []
    digests = []
    for s in srcs:
        o = BUILD / (s.name + ".o")
        objs.append(o)
        if s.suffix == ".hip":
            cmd = [_hipcc(), *HIP_FLAGS, "-x", "hip", *_py_includes(), "-c", str(s), "-o", str(o)]
        else:
            # host-only translation unit (pybind11 glue); still compiled by hipcc so
            # hip_runtime types resolve, but with no device code of its own.
            cmd = [_hipcc(), *HIP_FLAGS, *_py_includes(), "-c", str(s), "-o", str(o)]
        d = _digest([s, *hdrs, *cmd])
        digests.append(d)
        if force or _stale(o, d):
            todo.append((cmd, o, d))

    def _compile(job):
        cmd, o, d = job
        _run(cmd)
        _stamp(o, d)

    if todo:
        jobs = jobs or min(len(todo), max(1, (os.cpu_count() or 4) // 2))
        with cf.ThreadPoolExecutor(jobs) as ex:
            list(ex.map(_compile, todo))
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs),
           f"-L{ROCM / 'lib'}", "-lamdhip64", "-lrccl", "-o", str(target)]
    digest = _digest([*digests, *cmd])
    if force or todo or _stale(target, digest):
        _run(cmd)
        _check_kernel_stubs(target)
        _stamp(target, digest)
    return target


def _check_kernel_stubs(lib: Path) -> None:
    """A kernel the host pass did not emit leaves its launch stub undefined in the shared
    object (seen with hipcc for a template kernel whose body holds a lambda over a
    ``__shared__`` array); the library links, and only the GPU box's dlopen fails.  Refuse it
    here instead."""
    nm = shutil.which("nm")
    if not nm:
        return
    out = subprocess.run([nm, "-D", "--undefined-only", str(lib)], capture_output=True, text=True).stdout
    bad = [ln.split()[-1] for ln in out.splitlines() if "__device_stub__" in ln]
    if bad:
        lib.unlink()
        raise RuntimeError(f"{lib.name}: undefined kernel launch stubs {bad}")


def build_all(force: bool = False, only: str | None = None, jobs: int | None = None) -> list[Path]:
    out = []
    if only in (None, "cpu"):
        out.append(build_cpu(force))
    if only in (None, "hip"):
        out.append(build_hip(force, jobs))
    return out


def main(argv=None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", choices=["cpu", "hip"], default=None)
    ap.add_argument("--jobs", type=int, default=None)
    a = ap.parse_args(argv)
    for p in build_all(a.force, a.only, a.jobs):
        print(p)


if __name__ == "__main__":
    main()
