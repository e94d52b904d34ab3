"""Build an A/B variant of the product library with extra -D defines:

    python tools/build_variant.py w2 TB_MIN_WAVES=2 [--tus k_lines.hip,k_w2_lines.hip]

-> teku_amd/lib/variants/libtekubls_hip_w2.so; run it with TBLS_LIB=<path>.
--tus: recompile only these translation units (the rest from the main build).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

if __name__ == "__main__":
    args = sys.argv[2:]
    only = None
    if "--tus" in args:
        k = args.index("--tus")
        only = args[k + 1].split(",")
        args = args[:k] + args[k + 2:]
    print(ge.build_hip_lib(variant=sys.argv[1], defines=args, only=only))
