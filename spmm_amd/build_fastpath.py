"""Builds spmm_amd/lib/fastpath/spmm_fastpath.so (csrc/fastpath.cpp, a torch C++ extension
linked against libmi355_spgemm.so).  Run by `make fastpath` / __graft_entry__.build();
importing it never compiles (spmm_amd/_fastpath.py loads the prebuilt file)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def main():
    from torch.utils.cpp_extension import load
    out = os.path.join(HERE, "lib", "fastpath")
    os.makedirs(out, exist_ok=True)
    load(name="spmm_fastpath", sources=[os.path.join(HERE, "csrc", "fastpath.cpp")],
         extra_include_paths=[os.path.join(ROOT, "include")],
         extra_cflags=["-O2"],
         extra_ldflags=[f"-L{os.path.join(HERE, 'lib')}", "-lmi355_spgemm", "-Wl,-rpath,\\$$ORIGIN/.."],
         build_directory=out, verbose=False)
    print(os.path.join(out, "spmm_fastpath.so"))


if __name__ == "__main__":
    sys.exit(main())
