"""In-tree native build of ``distriflow_amd._C`` (HIP kernels for gfx950 + C++ runtime + bindings).

No JIT cache, no hipify: every ``csrc/*.hip`` file is compiled with ``hipcc --offload-arch=gfx950``
straight from source, ``csrc/*.cpp`` (bindings + host runtime) with hipcc as host C++, and the
objects are linked against PyTorch's own libraries into ``distriflow_amd/_C.so`` so that the
built module travels with the repository snapshot to the GPU box.

Incremental: an object is rebuilt when its source or any ``csrc/*.h`` header is newer.
Run ``python -m distriflow_amd._build [--force] [-v]``.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
OBJDIR = os.path.join(ROOT, "build", "obj")
OUT = os.path.join(ROOT, "distriflow_amd", "_C.so")
ARCH = os.environ.get("DISTRIFLOW_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_paths():
    import torch.utils.cpp_extension as ce

    return ce.include_paths(), ce.library_paths()


def _flags():
    incs, _ = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    common = [
        "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
        "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-D_GLIBCXX_USE_CXX11_ABI=1",
        "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
        "-Wno-unused-result", "-Wno-deprecated-declarations",
        f"-I{CSRC}", f"-I{py_inc}", "-I/opt/rocm/include",
    ] + [f"-I{i}" for i in incs]
    return common


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _obj_for(src):
    return os.path.join(OBJDIR, os.path.basename(src) + ".o")


def _needs(src, obj, hdr_mtime):
    if not os.path.exists(obj):
        return True
    om = os.path.getmtime(obj)
    return os.path.getmtime(src) > om or hdr_mtime > om


def _compile(src, obj, verbose):
    cmd = [HIPCC] + _flags() + ["-c", src, "-o", obj]
    if src.endswith(".cpp"):
        # host-only translation units: no device code, skip the device pass
        cmd = [HIPCC] + [f for f in _flags() if not f.startswith("--offload-arch")] + ["-x", "c++", "-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, verbose: bool = False, jobs: int | None = None) -> str:
    """Compile and link ``distriflow_amd/_C.so``; returns its path.

    ``DISTRIFLOW_SKIP_BUILD=1`` trusts an existing ``_C.so`` (e.g. a snapshot copied to a GPU box
    whose file mtimes were not preserved)."""
    if os.environ.get("DISTRIFLOW_SKIP_BUILD") == "1" and os.path.exists(OUT) and not force:
        return OUT
    os.makedirs(OBJDIR, exist_ok=True)
    srcs = _sources()
    hdrs = glob.glob(os.path.join(CSRC, "*.h"))
    hdr_mtime = max([os.path.getmtime(h) for h in hdrs] + [0.0])
    todo = [(s, _obj_for(s)) for s in srcs if force or _needs(s, _obj_for(s), hdr_mtime)]
    jobs = jobs or min(8, max(1, (os.cpu_count() or 4)))
    # the bindings TU (torch headers) is the slowest; start it first
    todo.sort(key=lambda so: 0 if "bindings" in so[0] else 1)
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            list(ex.map(lambda so: _compile(so[0], so[1], verbose), todo))
    objs = [_obj_for(s) for s in srcs]
    if todo or force or not os.path.exists(OUT) or max(os.path.getmtime(o) for o in objs) > os.path.getmtime(OUT):
        _, libs = _torch_paths()
        tmp = OUT + ".tmp"
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp]
        for d in libs:
            cmd += [f"-L{d}", f"-Wl,-rpath,{d}"]
        cmd += ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python", "-lamdhip64"]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    p = build(force="--force" in sys.argv, verbose="-v" in sys.argv)
    print(p)
