"""Source id of libmi355_spgemm.so: the first 16 hex digits of the SHA-256 over the sources
the library is compiled from (spmm_amd/csrc/*.hip, *.hpp, include/*.h: name and content,
sorted) and the effective HIPFLAGS.  The Makefile compiles it INTO the library
(spg_build_info); measurements (profiles/pmc_traffic.json) are stamped with the id the
loaded library reports, so an A/B build, a stale .so or a `make HIPFLAGS=...` variant never
matches numbers taken on another build.

usage: python3 spmm_amd/source_id.py '<HIPFLAGS>'
"""
import glob
import hashlib
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))


def compute(hipflags: str) -> str:
    root = os.path.dirname(_HERE)
    files = sorted(glob.glob(os.path.join(_HERE, "csrc", "*.hip")) + glob.glob(os.path.join(_HERE, "csrc", "*.hpp"))
                   + glob.glob(os.path.join(root, "include", "*.h")), key=os.path.basename)
    h = hashlib.sha256()
    for fn in files:
        h.update(os.path.basename(fn).encode())
        with open(fn, "rb") as f:
            h.update(f.read())
    h.update(" ".join(hipflags.split()).encode())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(compute(sys.argv[1] if len(sys.argv) > 1 else ""))
