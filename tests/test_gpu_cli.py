"""End-to-end drop-in CLIs on the GPU: the teacher CLI (train_teacher_gnn.py)
trains a SAGE teacher on a synthetic cora-shape graph and writes the
reference's artefacts, then the student CLI (main.py) distils from them in
full-batch and minibatch mode, printing the reference's result lines."""
import contextlib
import io
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture()
def workdir(tmp_path):
    w = tmp_path / "src"
    w.mkdir()
    old = os.getcwd()
    os.chdir(w)
    yield tmp_path
    os.chdir(old)


def _run(mod, argv):
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        mod.main(argv)
    return buf.getvalue()


def test_teacher_then_student_cli(workdir):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import main as student_cli
    import train_teacher_gnn as teacher_cli
    out = _run(teacher_cli, ["--datasets=cora", "--encoder=sage", "--runs=1", "--epochs=3", "--synthetic",
                             "--lr=0.005"])
    assert "Hits@20" in out and "Run: 01, Epoch: 03" in out and "All runs:" in out
    tag = "cora-sage_transductive.pkl"
    feats = torch.load(workdir / "saved-features" / tag, weights_only=True)["features"]
    sd = torch.load(workdir / "saved-models" / tag, weights_only=True)
    assert feats.shape == (2708, 256) and torch.isfinite(feats).all()
    assert set(sd) == {"gnn", "predictor"} and "convs.0.lin_l.weight" in sd["gnn"]
    # README command (README.md:26) shape, 2 epochs, full-batch train()
    out = _run(student_cli, ["--datasets=cora", "--encoder=sage", "--runs=1", "--epochs=2", "--synthetic",
                             "--KD_RM=0", "--LLP_D=0.001", "--KD_LM=0", "--LLP_R=1", "--True_label=0.1",
                             "--dropout=0.5", "--hops=2", "--lr=0.01", "--margin=0.1", "--ns_rate=1",
                             "--ps_method=nb", "--rw_step=3"])
    lines = [l for l in out.splitlines() if l.startswith("Run: 01, Epoch: 02")]
    assert len(lines) == 5, out          # Hits@10/20/30/50 + AUC
    assert "Loss: " in lines[0] and "Valid: " in lines[0] and "Test: " in lines[0]
    assert os.path.exists(workdir / "results" / "cora_KD_transductive.txt")
    # minibatch path (train_minibatch) with PyG-dense negatives, bf16 engine
    out = _run(student_cli, ["--datasets=cora", "--encoder=sage", "--runs=1", "--epochs=2", "--synthetic",
                             "--minibatch", "--LLP_D=1", "--LLP_R=1", "--True_label=1", "--dropout=0.0",
                             "--hops=2", "--rw_step=2", "--ns_rate=2", "--dtype=bf16", "--link_batch_size=1024"])
    assert "Run: 01, Epoch: 02" in out


def test_production_cli(workdir):
    """Production (inductive) setting end to end: the teacher CLI makes and
    caches the split (src/train_teacher_gnn.py:341-365), trains on the
    old-node graph and reports old_old / old_new / new_new; the student CLI
    reads the same split and the teacher's artefacts (src/main.py:337-346)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import main as student_cli
    import train_teacher_gnn as teacher_cli
    out = _run(teacher_cli, ["--datasets=cora", "--encoder=sage", "--runs=1", "--epochs=2", "--synthetic",
                             "--transductive=production"])
    assert "splitting the datasets now..." in out and "#Old Nodes:\t1896" in out
    line = [l for l in out.splitlines() if l.startswith("Run: 01, Epoch: 02")][0]
    for k in ("valid: ", "test: ", "old_old: ", "old_new: ", "new_new: "):
        assert k in line, line
    assert os.path.exists(workdir / "data" / "cora_production.pt")
    tag = "cora-sage_production.pkl"
    feats = torch.load(workdir / "saved-features" / tag, weights_only=True)["features"]
    assert feats.shape == (1896, 256) and torch.isfinite(feats).all()
    out = _run(student_cli, ["--datasets=cora", "--encoder=sage", "--runs=1", "--epochs=2", "--synthetic",
                             "--transductive=production", "--LLP_D=1", "--LLP_R=1", "--True_label=0.1",
                             "--dropout=0.0", "--hops=1", "--rw_step=3", "--ns_rate=1"])
    assert "splitting the datasets now..." not in out          # the cached split is reused
    lines = [l for l in out.splitlines() if l.startswith("Run: 01, Epoch: 02")]
    assert len(lines) == 5 and "new_new: " in lines[0], out
    txt = open(workdir / "results" / "cora_KD_production.txt").read()
    assert "Final old_new" in txt


def test_gcn_teacher_cli(workdir):
    """--encoder=gcn (src/train_teacher_gnn.py:384-387) writes the artefacts the
    student CLI reads under the gcn tag."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import train_teacher_gnn as teacher_cli
    out = _run(teacher_cli, ["--datasets=cora", "--encoder=gcn", "--runs=1", "--epochs=2", "--synthetic"])
    assert "Run: 01, Epoch: 02" in out
    sd = torch.load(workdir / "saved-models" / "cora-gcn_transductive.pkl", weights_only=True)
    assert "convs.0.lin.weight" in sd["gnn"] and "convs.0.bias" in sd["gnn"]
