"""morph() (R/morph.R:30-209, R/utilities_morph.R): the formula arithmetic on the
host (hand-derived expectations from the R source; parity unpinned against R
itself, which is absent) and, on the GPU, the nMorphs soundgen() calls run as
one batch with the same bytes as calling soundgen() on each formula."""
import math

import numpy as np
import pytest

from soundgen_beta_amd import morph as M
from soundgen_beta_amd import presets


def test_morphDF_per_anchor_hand_case():
    # a = data.frame(0:1, .5) (soundgen's mouthAnchors default), b with a middle anchor:
    # b is longer -> swapped; the middle anchor (.5, 1 normalised) is equidistant from
    # both ends of a and takes the first; hybrid d: row + idx[d] * (match - row)
    a = M.DataFrame(time=[0.0, 1.0], value=[.5, .5])
    b = {"time": [0, .5, 1], "value": [0, .5, 0]}
    out = M.morphDF(a, b, 5)
    assert out[0] == {"time": [0.0, 1.0], "value": [.5, .5]}  # d = 5 after the swap, duplicates removed
    assert out[2] == {"time": [0.0, .25, 1.0], "value": [.25, .5, .25]}
    assert out[4] == {"time": [0.0, .5, 1.0], "value": [0.0, .5, 0.0]}


def test_morphDF_identical_and_na():
    a = {"time": [0, 1], "value": [1, 2]}
    assert M.morphDF(a, dict(a), 3) == [a, a, a]
    # NA on one side: the other side's times with zero values
    out = M.morphDF(None, {"time": [0, 1], "value": [10, 20]}, 3)
    assert out[0] == {"time": [0.0, 1.0], "value": [0.0, 0.0]} and out[1] == {"time": [0.0, 1.0], "value": [5.0, 10.0]}


def test_morphList_equalises_formant_counts_with_silent_copies():
    l1 = {"f1": {"time": 0, "freq": 700, "amp": 30, "width": 80},
          "f2": {"time": 0, "freq": 900, "amp": 30, "width": 120},
          "f3": {"time": 0, "freq": 1500, "amp": 20, "width": 150}}
    l2 = {"f1": {"time": 0, "freq": 400, "amp": 40, "width": 120}}
    out = M.morphList(l1, l2, 3)
    assert len(out) == 3 and list(out[0]) == ["f1", "f2", "f3"]
    # f2 of l2 is l1's f2 silenced: amplitude morphs 30 -> 0, frequency stays
    assert out[1]["f2"]["amp"] == [15.0, 15.0] and out[1]["f2"]["freq"] == [900.0, 900.0]
    assert out[2]["f1"]["freq"] == [400.0, 400.0] and out[0]["f1"]["freq"] == [700.0, 700.0]


def test_morphList_l2_longer_names_by_position():
    """R/utilities_morph.R:261-265: when l2 is longer, l1 grows and the new slot is
    named names(l2)[length(l1)] AFTER the append, i.e. l2's name at that position."""
    l1 = {"f1": {"time": 0, "freq": 700, "amp": 30, "width": 80}}
    l2 = {"f1": {"time": 0, "freq": 400, "amp": 40, "width": 120},
          "f2": {"time": 0, "freq": 1100, "amp": 30, "width": 120},
          "f3": {"time": 0, "freq": 2500, "amp": 20, "width": 150}}
    out = M.morphList(l1, l2, 3)
    assert list(out[0]) == ["f1", "f2", "f3"]
    assert out[0]["f2"]["amp"] == [0.0, 0.0] and out[2]["f2"]["amp"] == [30.0, 30.0]
    # an empty l1 becomes l2's formants silenced, named f1, f2, f3 (formants$f1 exists)
    out = M.morphList({}, l2, 2)
    assert list(out[0]) == ["f1", "f2", "f3"] and out[0]["f1"]["amp"] == [0.0, 0.0]


def test_morph_formulas_roxygen_example():
    """morph(formula1 = list(repeatBout = 2), formula2 = presets$Misc$Dog_bark, nMorphs = 5):
    non-default pars of either side are morphed; scalars by seq(), pitch in log Hz."""
    f2 = presets.args("Misc", "Dog_bark")
    fs = M.morph_formulas({"repeatBout": 2}, f2, 5)
    assert len(fs) == 5 and all(list(f) == list(fs[0]) for f in fs)
    assert [f["sylLen"] for f in fs] == [300.0, 260.0, 220.0, 180.0, 140.0]  # seq(300, 140, length.out = 5)
    assert all(f["repeatBout"] == 2.0 for f in fs)  # Dog_bark has repeatBout 2
    p0, p4 = fs[0]["pitchAnchors"], fs[4]["pitchAnchors"]
    assert np.allclose(p0["value"], [100, 150, 135, 100], rtol=1e-14)  # exp(log(x)) round trip
    assert np.allclose(p4["value"], f2["pitchAnchors"]["value"], rtol=1e-14)
    # geometric interpolation of the middle pitch: exp(mean of logs) of matched anchors
    assert math.isclose(fs[2]["pitchAnchors"]["value"][0], math.sqrt(100 * 559), rel_tol=1e-12)
    # the string form of a formula parses to the same list
    fs2 = M.morph_formulas("soundgen(repeatBout = 2)", f2, 5)
    assert fs2 == fs


@pytest.mark.gpu
def test_morph_batch_equals_single_calls(tmp_path):
    from soundgen_beta_amd import api
    rng = np.random.default_rng(3)
    Z, U = rng.standard_normal(100000), rng.uniform(size=2000000)
    m = M.morph({"repeatBout": 2}, presets.args("Misc", "Dog_bark"), 5, samplingRate=16000, normals=Z, uniforms=U,
                savePath=str(tmp_path) + "/")
    for f, y in zip(m["formulas"], m["sounds"]):
        ref = api.soundgen(normals=Z, uniforms=U, **M._soundgen_args(f))
        assert len(ref) == len(y) and np.array_equal(np.float32(ref), np.float32(y))
    for h in range(5):
        assert (tmp_path / ("morph_%d.wav" % (h + 1))).stat().st_size == 80 + 2 * len(m["sounds"][h])
    # per-morph draws (R's one stream split at the morph boundaries): morph h reads its own arrays
    Zs = [Z[h * 1000:] for h in range(5)]
    m2 = M.morph({"repeatBout": 2}, presets.args("Misc", "Dog_bark"), 5, samplingRate=16000, normals=Zs, uniforms=U)
    for h, (f, y) in enumerate(zip(m2["formulas"], m2["sounds"])):
        ref = api.soundgen(normals=Zs[h], uniforms=U, **M._soundgen_args(f))
        assert len(ref) == len(y) and np.array_equal(np.float32(ref), np.float32(y))
