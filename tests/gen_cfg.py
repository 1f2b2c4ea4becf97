"""The reference's benchmark env configs (the same builders tools/gen_fixtures.py uses)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
from gen_fixtures import div1, div2, serial4, serial8  # noqa: E402,F401
