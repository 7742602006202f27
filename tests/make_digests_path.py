"""puts tests/golden on sys.path (for importing make_digests in tests)"""
import os
import sys

_G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
if _G not in sys.path:
    sys.path.insert(0, _G)
