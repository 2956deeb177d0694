"""In-tree build of the native extension ``commefficient_amd/_C.so``.

* ``csrc/*.hip``  -> hipcc ``--offload-arch=gfx950`` (device kernels + launchers,
  no torch headers, so each file compiles in seconds);
* ``csrc/*.cpp``  -> g++ with the torch + HIP headers (op registration and the
  native CPU backend);
* link into one shared object that ``torch.ops.load_library`` loads.  The HIP
  runtime is resolved against the copy torch already loaded (same SONAME).

Run ``python -m commefficient_amd.build`` (or ``__graft_entry__.build()``).
Incremental: an object is rebuilt when its source or any header is newer.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(os.path.dirname(PKG), "build", "obj")
OUT = os.path.join(PKG, "_C.so")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def _torch_paths():
    import torch
    root = os.path.dirname(torch.__file__)
    inc = [os.path.join(root, "include"),
           os.path.join(root, "include", "torch", "csrc", "api", "include")]
    return inc, os.path.join(root, "lib"), torch._C._GLIBCXX_USE_CXX11_ABI


def _newer(src: str, obj: str, headers) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return os.path.getmtime(src) > t or any(os.path.getmtime(h) > t for h in headers)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def build(verbose: bool = False, force: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    inc, tlib, cxx11 = _torch_paths()
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    hip_srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    cpp_srcs = sorted(glob.glob(os.path.join(CSRC, "*.cpp")))
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    py_inc = sysconfig.get_paths()["include"]

    jobs = []
    for s in hip_srcs:
        o = os.path.join(OBJ, os.path.basename(s) + ".o")
        if force or _newer(s, o, headers):
            jobs.append([hipcc, "-c", "-fPIC", "-O3", "-std=c++17", f"--offload-arch={ARCH}",
                         "-munsafe-fp-atomics", "-Wall", "-I", CSRC, s, "-o", o])
    abi = f"-D_GLIBCXX_USE_CXX11_ABI={int(cxx11)}"
    for s in cpp_srcs:
        o = os.path.join(OBJ, os.path.basename(s) + ".o")
        if force or _newer(s, o, headers):
            cmd = ["g++", "-c", "-fPIC", "-O3", "-std=c++17", "-fopenmp", abi,
                   "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=_C",
                   "-I", CSRC, "-I", os.path.join(ROCM, "include"), "-I", py_inc]
            for i in inc:
                cmd += ["-isystem", i]
            jobs.append(cmd + [s, "-o", o])
    nproc = int(os.environ.get("MAX_JOBS", min(8, os.cpu_count() or 4)))
    with cf.ThreadPoolExecutor(max_workers=nproc) as ex:
        for out in ex.map(_run, jobs):
            if verbose and out.strip():
                print(out)
    objs = [os.path.join(OBJ, os.path.basename(s) + ".o") for s in hip_srcs + cpp_srcs]
    if force or jobs or not os.path.exists(OUT) or any(
            os.path.getmtime(o) > os.path.getmtime(OUT) for o in objs):
        link = ["g++", "-shared", "-o", OUT + ".tmp"] + objs + [
            "-L", tlib, "-Wl,-rpath," + tlib, "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch_hip",
            "-ltorch", "-L", os.path.join(ROCM, "lib"), "-lamdhip64", "-fopenmp"]
        _run(link)
        os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    p = build(verbose="-v" in sys.argv, force="--force" in sys.argv)
    print("built", p)
