"""Per-kernel register / LDS / spill summary of one gfx950 HIP source (hipcc -Rpass-analysis=kernel-resource-usage).

usage: python scripts/kernel_resources.py csrc/attention.hip [--filter attn_bwd] [-- extra clang flags]
Run it after every edit of a hand-scheduled kernel: a VGPR spill or a scratch size > 0 is a bug."""
import os
import re
import subprocess
import sys


def main():
    args = sys.argv[1:]
    extra = []
    if "--" in args:
        k = args.index("--")
        args, extra = args[:k], args[k + 1:]
    src = args[0]
    flt = args[args.index("--filter") + 1] if "--filter" in args else ""
    inc = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pretraining_llm_amd", "csrc")
    cmd = ["/opt/rocm/lib/llvm/bin/clang++", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
           "-munsafe-fp-atomics", "-c", "-x", "hip", src, "-I", inc, "-o", "/tmp/_kres.o", "--offload-device-only",
           "-Rpass-analysis=kernel-resource-usage"] + extra
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    cur, rows = None, []
    for line in out.splitlines():
        m = re.search(r"remark:\s+Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+)", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = int(m.group(2))
    print(f"{'kernel':70s} {'VGPR':>5s} {'AGPR':>5s} {'VSpill':>6s} {'SSpill':>6s} {'LDS':>7s} {'occ':>3s}")
    for r in rows:
        n = re.sub(r"^_ZN12_GLOBAL__N_1\d+", "", r["name"])
        if flt and flt not in n:
            continue
        print(f"{n[:70]:70s} {r.get('VGPRs', 0):5d} {r.get('AGPRs', 0):5d} {r.get('VGPRs Spill', 0):6d} "
              f"{r.get('SGPRs Spill', 0):6d} {r.get('LDS Size', 0):7d} {r.get('Occupancy', 0):3d}")
    if "error" in out:
        print(out[-3000:])


if __name__ == "__main__":
    main()
