"""CLI entry of the configs[0] runner (s2v_amd.inference; the package directory name has hyphens):

    python tools/run_inference.py --face examples/face/1.mp4 --audio examples/audio/1.wav --max_frames 8
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import s2v_import  # noqa: E402,F401
from s2v_amd import inference  # noqa: E402

if __name__ == "__main__":
    sys.exit(inference.main())
