"""PVR probe correctness / leakiness per conv hook point (parity: ``/root/reference/eval_information.py``).

Entry point kept at the repository root (the reference's script path); the implementation lives in
``iit_amd/entry/eval_information.py`` so an installed package provides it too (``python -m iit_amd.entry.eval_information``).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from iit_amd.entry.eval_information import *  # noqa: E402,F401,F403  (module-level names, e.g. for tests)
from iit_amd.entry.eval_information import main  # noqa: E402

if __name__ == "__main__":
    main()
