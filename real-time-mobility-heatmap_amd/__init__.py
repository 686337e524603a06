"""Package directory of the MI355X-native hot path (csrc/ = HIP kernels + C ABI, mobheat/ = host mirror).

The directory name is not a Python identifier; callers put this directory on sys.path and ``import mobheat``.
"""
import os
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
if PKG_DIR not in sys.path:
    sys.path.insert(0, PKG_DIR)
