#!/usr/bin/env python3
"""__graft_entry__.smoke() without the build step (the box runs the prebuilt
in-tree libraries): one small batch decode on cuda:0 against the oracle."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    import __graft_entry__

    __graft_entry__.smoke()
