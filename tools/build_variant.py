"""Build an A/B variant of the product library with extra -D defines:

    python tools/build_variant.py w2 TB_MIN_WAVES=2

-> teku_amd/lib/variants/libtekubls_hip_w2.so; run it with TBLS_LIB=<path>.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402

if __name__ == "__main__":
    print(ge.build_hip_lib(variant=sys.argv[1], defines=sys.argv[2:]))
