"""C5 pruned loop with and without SharedModel.note_selections (selections
joining the dedup set at round time): `python c5_note_ab.py off|on`."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from uptune_amd import technique as T  # noqa: E402

if sys.argv[1] == "off":
    T.SharedModel.note_selections = lambda self, hexes: None
sys.argv = [sys.argv[0], "--generations", "100", "--prune", "256"]
from scripts.c5_bandit import main  # noqa: E402

main()
