"""Link an A/B build of the extension: every kernel object as in the normal build, except
csrc/<file> compiled with extra flags (e.g. -D switches of an experiment).  Select it at run
time with PLLM_SO=<out> (ops/_lib.py).

usage: python scripts/build_variant.py attention.hip out.so [--from other.hip] [-DFOO=1 ...]
(--from: compile another version of that file instead, e.g. `git show HEAD~1:...` output)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pretraining_llm_amd import build as B  # noqa: E402


def main():
    src_name, out, *flags = sys.argv[1:]
    src_path = os.path.join(B.CSRC, src_name)
    if flags[:1] == ["--from"]:
        src_path, flags = os.path.abspath(flags[1]), flags[2:]
    B.build()  # normal objects up to date
    hipcc = B._hipcc()
    _, lib, _ = B._torch_paths()
    tag = os.path.splitext(os.path.basename(out))[0]
    vobj = os.path.join(B.BUILD, f"{src_name}.{tag}.o")
    B._run([hipcc, *B.COMMON_FLAGS, *B.FILE_FLAGS.get(src_name, []), *flags, "-I", B.CSRC, "-c", src_path,
            "-o", vobj])
    import glob
    names = [os.path.basename(p) + ".o" for p in sorted(glob.glob(os.path.join(B.CSRC, "*.hip")))]
    # every torch-facing translation unit (bindings.cpp, blaslt.cpp, ...), as the normal build links them
    names += [os.path.splitext(os.path.basename(p))[0] + ".o" for p in sorted(glob.glob(os.path.join(B.CSRC, "*.cpp")))]
    objs = [vobj if n == f"{src_name}.o" else os.path.join(B.BUILD, n) for n in names]
    B._run([hipcc, "-shared", f"--offload-arch={B.ARCH}", *objs, "-o", out, f"-L{lib}", "-lc10", "-lc10_hip", "-ltorch",
            "-ltorch_cpu", "-ltorch_hip", "-lhipblaslt", f"-Wl,-rpath,{lib}"])
    print(out)


if __name__ == "__main__":
    main()
