"""Check built gfx950 code objects for the long-branch / return-address hazard.

When a function's branch spans more than the short-branch range (+-2^16
words), the compiler expands it into s_getpc_b64 / s_add_u32 / s_addc_u32 /
s_setpc_b64 through a scratch SGPR pair.  In an outlined (non-kernel) function
ROCm 7.2's clang picked s[30:31] -- the return address -- for that pair
without saving it, so the function's return jumped back into itself and the
wave never finished (round 4: jac_mul_xabs_nx as an outlined 270 KB loop hung
the GPU).  This lists every non-kernel function whose code writes s[30:31]
with s_getpc_b64 (a function never needs to: its return address arrives in
s[30:31]).

    python tools/check_long_branches.py [lib.so | obj.o ...]   (exit 1 on a finding)
"""

import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def code_objects(path, d):
    """gfx950 code objects inside a host object / shared library's .hip_fatbin."""
    fb = os.path.join(d, os.path.basename(path) + ".fatbin")
    if subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", path, os.path.join(d, "junk")],
                      capture_output=True).returncode:
        return []
    out = []
    # a fatbin may hold several bundles (one per TU in a shared library): split on the bundle magic
    blob = open(fb, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), blob)] or [0]
    for k, st in enumerate(starts):
        end = starts[k + 1] if k + 1 < len(starts) else len(blob)
        part = os.path.join(d, f"{os.path.basename(path)}.{k}.bundle")
        with open(part, "wb") as f:
            f.write(blob[st:end])
        co = part + ".co"
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={part}",
                            f"--output={co}", "--unbundle"], capture_output=True)
        if r.returncode == 0 and os.path.getsize(co) > 0:
            out.append(co)
    return out


def findings(co):
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], capture_output=True, text=True).stdout
    syms = subprocess.run([f"{LLVM}/llvm-readelf", "-s", "-W", co], capture_output=True, text=True).stdout
    kernels = {l.split()[-1][:-3] for l in syms.splitlines() if l.split() and l.split()[-1].endswith(".kd")}
    bad, cur = set(), None
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = m.group(1)
            continue
        if cur and cur not in kernels and re.search(r"s_getpc_b64\s+s\[30:31\]", line):
            bad.add(cur)
    return sorted(bad)


def main(paths):
    paths = paths or [os.path.join(ROOT, "teku_amd", "lib", "libtekubls_hip.so")]
    found = []
    with tempfile.TemporaryDirectory() as d:
        for p in paths:
            for co in code_objects(p, d):
                found += [(p, f) for f in findings(co)]
    for p, f in found:
        print(f"{os.path.relpath(p, ROOT)}: {f}: long branch through s[30:31] (the return address)")
    return 1 if found else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
