"""Build the in-tree gfx950 HIP extension ``pretraining_llm_amd/_C.so``.

No hipify, no ``torch.utils.cpp_extension`` JIT: every ``csrc/*.hip`` kernel file
is compiled straight for ``--offload-arch=gfx950`` by ``hipcc`` (kernel files
include only ``hip_runtime.h`` so they compile in seconds), ``bindings.cpp``
(the only file that sees torch headers) registers the ops under
``torch.ops.pllm``, and everything is linked against the torch/HIP libraries
that ship with the installed PyTorch-ROCm.  Objects are cached under
``csrc/build`` and rebuilt when a source or header changes.

Usage: ``python -m pretraining_llm_amd.build [--force] [-j N] [--debug]``

``--debug`` rebuilds everything with ``-DPLLM_DEBUG``: the kernels then report contract
violations they otherwise tolerate silently (out-of-range token ids / targets) with a device
printf naming the kernel and the offending value (no trap: a faulting kernel can take the
whole node down).  Combine with ``debug_sync=True`` in the trainer config
(AMD_SERIALIZE_KERNEL=3 + HIP_LAUNCH_BLOCKING=1) to attribute a failure to one launch.
Rebuild with ``--force`` to return to the release objects.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(CSRC, "build")
OUT = os.path.join(HERE, "_C.so")
HOST_OUT = os.path.join(HERE, "_host.so")
ARCH = os.environ.get("PLLM_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build the gfx950 extension)")


def _torch_paths():
    import torch
    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    lib = os.path.join(tdir, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


COMMON_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
                "-Wno-unused-result", "-Wno-unused-variable"]


# per-file flags.  attention.hip: no SLP vectorisation -- it packs pairs of independent f32
# multiplies of the softmax / dS math into v_pk_mul_f32 plus two v_mov each to gather the
# operands, more vector issue beside the MFMAs than the scalar multiplies
FILE_FLAGS = {"attention.hip": ["-fno-slp-vectorize"], "attn_bwd_ks.hip": ["-fno-slp-vectorize"]}


def _needs(obj: str, deps) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def build_host(force: bool = False) -> str:
    """Host-side native runtime (token loader): plain C++17, no GPU, no torch."""
    srcs = sorted(glob.glob(os.path.join(CSRC, "host", "*.cpp")))
    if force or _needs(HOST_OUT, srcs):
        cxx = os.environ.get("CXX", shutil.which("g++") or shutil.which("c++") or "g++")
        _run([cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", *srcs, "-o", HOST_OUT + ".tmp"])
        os.replace(HOST_OUT + ".tmp", HOST_OUT)
    return HOST_OUT


def build(force: bool = False, jobs: int = 8, verbose: bool = False, debug: bool = False) -> str:
    global COMMON_FLAGS
    if debug:
        force = True
        COMMON_FLAGS = COMMON_FLAGS + ["-DPLLM_DEBUG=1"]
    build_host(force)
    os.makedirs(BUILD, exist_ok=True)
    hipcc = _hipcc()
    inc, lib, abi = _torch_paths()
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    kernel_srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    bind_src = os.path.join(CSRC, "bindings.cpp")
    jobs_list = []
    for src in kernel_srcs:
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        cmd = [hipcc, *COMMON_FLAGS, *FILE_FLAGS.get(os.path.basename(src), []), "-c", src, "-o", obj]
        jobs_list.append((obj, [src, *headers], cmd))
    # torch-facing translation units: bindings.cpp (op registration) and blaslt.cpp (hipBLASLt epilogues)
    py_inc = sysconfig.get_paths()["include"]
    for src in [bind_src] + sorted(p for p in glob.glob(os.path.join(CSRC, "*.cpp")) if p != bind_src):
        bobj = os.path.join(BUILD, os.path.splitext(os.path.basename(src))[0] + ".o")
        bcmd = [hipcc, *COMMON_FLAGS, "-c", "-x", "hip", src, "-o", bobj, f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
                "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1", *[f"-I{p}" for p in inc], f"-I{py_inc}"]
        jobs_list.append((bobj, [src, *headers], bcmd))
    todo = [(o, c) for (o, d, c) in jobs_list if force or _needs(o, d)]
    if todo:
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            futs = {ex.submit(_run, c): o for (o, c) in todo}
            for f in cf.as_completed(futs):
                out = f.result()
                if verbose and out.strip():
                    print(out)
    objs = [o for (o, _, _) in jobs_list]
    if force or todo or _needs(OUT, objs):
        lcmd = [hipcc, "-shared", f"--offload-arch={ARCH}", *objs, "-o", OUT + ".tmp", f"-L{lib}", "-lc10", "-lc10_hip",
                "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-lhipblaslt", f"-Wl,-rpath,{lib}"]
        _run(lcmd)
        os.replace(OUT + ".tmp", OUT)
    return OUT


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=int(os.environ.get("MAX_JOBS", "8")))
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--debug", action="store_true", help="device-side contract diagnostics (-DPLLM_DEBUG)")
    args = ap.parse_args(argv)
    out = build(force=args.force, jobs=args.jobs, verbose=args.verbose, debug=args.debug)
    print(out)


if __name__ == "__main__":
    sys.exit(main())
