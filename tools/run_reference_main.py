#!/usr/bin/env python3
"""Run the reference's own, unchanged main.py on the MI355X drop-in (nfsp_amd.reference_main):

    python tools/run_reference_main.py /path/to/reference/main.py [--episodes N] [-- main.py args]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    pkg = __import__("__graft_entry__").load_package()
    sys.exit(pkg.reference_main.main())
