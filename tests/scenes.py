"""test-side shim: scene paths come from the product's scene resolver (prt.scenes)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parallel-ray-tracer_amd"))
from prt.scenes import scene_paths  # noqa: E402,F401
