"""presets$<speaker>$<name> of the reference (R/presets.R:156-410): the soundgen()
argument sets, as data (presets.json, written by tools/extract_presets.py).

    from soundgen_beta_amd import presets, soundgen
    y = soundgen(**presets.args("M1", "Gasp"))
"""
import copy
import json
import os

_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "presets.json")
_DATA = None


def _data():
    global _DATA
    if _DATA is None:
        with open(_PATH) as f:
            _DATA = json.load(f)
    return _DATA


def speakers():
    return sorted(_data())


def names():
    """[(speaker, preset)] in a fixed order."""
    return [(s, n) for s in speakers() for n in sorted(_data()[s])]


def args(speaker, name):
    """The preset's soundgen() arguments (a fresh copy; R names)."""
    return copy.deepcopy(_data()[speaker][name])
