"""Per-kernel register / scratch / LDS usage of the built kernels, read from the
gfx950 code objects' AMDGPU metadata of the per-TU objects (no GPU needed):

    python tools/kernel_resources.py [teku_amd/lib/obj/*.o]

The unified VGPR+AGPR count per lane (.vgpr_count; .agpr_count of them are
AGPRs) sets the waves per SIMD (MI355X_MICROARCH.md, register files: <=128 ->
4, <=168 -> 3, <=256 -> 2, else 1); private_segment_fixed_size is the scratch
(spill) bytes per lane.
"""

import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def waves_per_simd(regs):
    for lim, w in [(64, 8), (72, 7), (80, 6), (96, 5), (128, 4), (168, 3), (256, 2), (512, 1)]:
        if regs <= lim:
            return w
    return 0


def main():
    import glob

    objs = sys.argv[1:] or sorted(glob.glob(os.path.join(os.path.dirname(__file__), "..", "teku_amd", "lib", "obj", "*.o")))
    rows = []
    with tempfile.TemporaryDirectory() as d:
        cos = []
        for k, o in enumerate(objs):
            fb, co = os.path.join(d, f"{k}.fatbin"), os.path.join(d, f"{k}.co")
            if subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", o, os.path.join(d, "junk")],
                              capture_output=True).returncode:
                continue
            subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                                   f"--input={fb}", f"--output={co}", "--unbundle"])
            cos.append(co)
        for co in cos:
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
            for blk in re.split(r"\n  - \.agpr_count:", notes)[1:]:  # one kernel entry each (keys sorted, .agpr_count first)
                blk = ".agpr_count:" + blk
                m = re.search(r"\n    \.name:\s+(\S+)", blk)
                if not m:
                    continue
                name = m.group(1)
                get = lambda k: int(re.search(rf"(?:^|\n    )\.{k}:\s+(\d+)", blk).group(1)) if re.search(rf"(?:^|\n    )\.{k}:\s+(\d+)", blk) else 0  # noqa: E731
                v, a = get("vgpr_count"), get("agpr_count")
                # gfx950's unified register file: .vgpr_count already includes the .agpr_count AGPRs
                rows.append((name, v, a, get("private_segment_fixed_size"), get("group_segment_fixed_size"), waves_per_simd(v)))
    print(f"{'kernel':32s} {'vgpr':>5s} {'agpr':>5s} {'scratch':>8s} {'lds':>7s} {'waves/SIMD':>10s}")
    for r in sorted(set(rows)):
        if r[0].endswith(".kd"):
            continue
        print(f"{r[0]:32s} {r[1]:5d} {r[2]:5d} {r[3]:8d} {r[4]:7d} {r[5]:10d}")


if __name__ == "__main__":
    main()
