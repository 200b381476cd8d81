#!/usr/bin/env python3
"""cupy_cusparse/gen_and_save_alg3_txt.py: gen_and_save_txt.py with --alg 3 fixed."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_and_save_txt import main  # noqa: E402

if __name__ == "__main__":
    main(alg=3)
