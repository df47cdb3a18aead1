"""The drop-in model classes keep the reference's constructor signatures
(src/models.py:7-15,57-58,83-84,122-123; src/sageconv_updated.py:39-42) and state_dict
keys and shapes, so checkpoints written by either side load in the other
(`../saved-models/*.pkl`, src/train_teacher_gnn.py:451-452, read at src/main.py:356-363).
Fixtures: tests/golden/api_signatures.json (tests/golden/gen_api_signatures.py) and the
reference-generated golden vectors, whose parameter keys are the reference modules'
own state_dict keys.  CPU only (construction; no forward)."""
import inspect
import json
import os

import pytest

import llp_sage
import models
from golden_io import load

HERE = os.path.dirname(os.path.abspath(__file__))
SIG = json.load(open(os.path.join(HERE, "golden", "api_signatures.json")))
OURS = {"MLP": models.MLP, "GCN": models.GCN, "SAGE": models.SAGE, "LinkPredictor": models.LinkPredictor,
        "SAGEConv_updated": llp_sage.SAGEConv_updated}


@pytest.mark.parametrize("name", sorted(SIG))
def test_constructor_signature(name):
    ps = list(inspect.signature(OURS[name].__init__).parameters.values())[1:]   # without self
    ours = [p for p in ps if p.kind not in (p.VAR_KEYWORD, p.VAR_POSITIONAL)]
    ref = SIG[name]["params"]
    assert [p.name for p in ours[:len(ref)]] == [p["name"] for p in ref]
    for p, r in zip(ours, ref):
        if "default" in r:
            assert p.default == r["default"], (name, p.name)
        else:
            assert p.default is inspect.Parameter.empty, (name, p.name)
    assert all(p.default is not inspect.Parameter.empty for p in ours[len(ref):]), "extra params must be optional"
    if SIG[name]["kwargs"]:
        assert any(p.kind == p.VAR_KEYWORD for p in ps), name


def _shapes(z, prefix):
    return {k[len(prefix):]: tuple(z[k].shape) for k in z.files if k.startswith(prefix)
            and (k.endswith(".weight") or k.endswith(".bias"))}


def _ours(module):
    return {k: tuple(v.shape) for k, v in module.state_dict().items()}


def test_mlp_and_predictor_state_dicts():
    z = load("models_fwd_bwd")
    ref = _shapes(z, "mlp/")
    ref = {k: v for k, v in ref.items() if not k.startswith("grad/")}
    L = len(ref) // 2
    m = models.MLP(L, ref["layers.0.weight"][1], ref["layers.0.weight"][0], ref[f"layers.{L - 1}.weight"][0], 0.0)
    assert _ours(m) == ref
    refp = {k: v for k, v in _shapes(z, "lp_mlp/").items() if not k.startswith("grad/")}
    Lp = len(refp) // 2
    lp = models.LinkPredictor("mlp", refp["lins.0.weight"][1], refp["lins.0.weight"][0],
                              refp[f"lins.{Lp - 1}.weight"][0], Lp, 0.0)
    assert _ours(lp) == refp


@pytest.mark.parametrize("case,conv", [("teacher_sage_small", "sage"), ("teacher_sage3_collab_small", "sage"),
                                       ("teacher_updated_production_small", "updated"),
                                       ("teacher_gcn_small", "gcn"), ("teacher_gcn3_production_small", "gcn")])
def test_teacher_state_dicts(case, conv):
    z = load(case)
    enc, pred = _shapes(z, "init/enc/"), _shapes(z, "init/pred/")
    L = len({k.split(".")[1] for k in enc})
    if conv == "gcn":
        w0, wl = enc["convs.0.lin.weight"], enc[f"convs.{L - 1}.lin.weight"]
        m = models.GCN(w0[1], w0[0], wl[0], L, 0.0)
    else:
        w0, wl = enc["convs.0.lin_l.weight"], enc[f"convs.{L - 1}.lin_l.weight"]
        layer = llp_sage.SAGEConv_updated if conv == "updated" else llp_sage.SAGEConv
        m = models.SAGE("collab", w0[1], w0[0], wl[0], L, 0.0, layer)
    assert _ours(m) == enc
    Lp = len(pred) // 2
    lp = models.LinkPredictor("mlp", pred["lins.0.weight"][1], pred["lins.0.weight"][0],
                              pred[f"lins.{Lp - 1}.weight"][0], Lp, 0.0)
    assert _ours(lp) == pred
