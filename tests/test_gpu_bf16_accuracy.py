"""bf16 training accuracy against fp32 (BASELINE north_star: Hits@20 within 0.1 of the
reference, which trains in fp32; src/main.py:379-385 collab metric keys).

Scaled synthetic ogbl-collab (tools/bf16_accuracy.py: scale 0.1, 2,000 planted
communities, so about five same-community pairs sit among the 10,000 random negatives and
Hits@20 measures link structure), the collab script's configuration at a 8,192-edge link
batch, 48 epochs.  fp32 and bf16 train from the same initial weights on the same
permutations and device draws; each model is evaluated through the device eval path in
fp32.  Each run is scored as the reference's Logger reports a run (Highest Valid, and
Final Test at that checkpoint, src/logger.py), and the statistic is the PAIRED per-seed
difference bf16 - fp32 over 8 seeds: |mean| + 2 SE.  Measured on MI355X
(profiles/r04_bf16_accuracy_paired.jsonl): Hits@20 +0.06 +- 0.31 pp (valid), +0.44 +- 0.47
(test); Hits@50 -0.05 +- 0.19, -0.25 +- 0.22 -- bounds 0.42-1.38 pp, against the fp32 runs'
own seed-to-seed SD of 1.2 pp (Hits@20 valid).  Both dtypes show the same transient loss
spikes late in training; a mean over the last checkpoints instead of the Logger's rule
catches them at random (bounds ~3 pp).  The unit of north_star's +-0.1: DESIGN.md §3."""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))


SEEDS = 8
# north_star's "Hits@20 within +-0.1 of reference" read in the unit the reference computes Hits@K
# in (the ogb Evaluator's fraction, src/train_teacher_gnn.py:121-143; the Logger prints x100):
# 0.1 = 10 percentage points.  DESIGN.md §3 gives the measured paired statistic and why the
# 0.1-pp reading is below what any seed count here can resolve (the fp32 runs' own seed-to-seed
# SD is ~2 pp).
BAR_PP = 10.0
GUARD_PP = 2.5   # a regression guard well inside it: the measured bounds are 0.4-1.4 pp (8 seeds)


def test_bf16_training_hits_track_fp32():
    """Paired over SEEDS seeds (bf16 and fp32 share init, permutations and draws, so the
    per-seed difference is the statistic), each run scored as the reference's Logger reports it
    (Highest Valid, and Final Test at that checkpoint): |mean(bf16 - fp32)| + 2 SE <= BAR_PP
    (and <= GUARD_PP) for Hits@20 and Hits@50 (tools/bf16_accuracy.py paired())."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import bf16_accuracy
    runs = [bf16_accuracy.compare(0.1, 8192, 48, seed=s, eval_every=8, communities=2000) for s in range(SEEDS)]
    for k in ("Hits@20", "Hits@50"):
        summ = bf16_accuracy.paired(runs, k, rule="best_valid")
        print(k, {sp: {q: summ[sp][q] for q in ("mean_pp", "se_pp", "bound_pp", "fp32_seed_sd_pp", "diff_pp")}
                  for sp in summ}, flush=True)
        for split in ("valid", "test"):
            st = summ[split]
            assert st["fp32_mean_pp"] > 60.0, (k, split, st)        # the models learned the link structure
            assert st["bound_pp"] <= BAR_PP and st["bound_pp"] <= GUARD_PP, (k, split, st)
    for r in runs:   # the training losses track each other (epochs 8-24; the overfitting onset varies by run)
        lf = [h["loss"] for h in r["runs"]["fp32"]["history"]]
        lb = [h["loss"] for h in r["runs"]["bf16"]["history"]]
        assert all(abs(a - b) <= 0.10 * a for a, b in zip(lf[:3], lb[:3])), (lf, lb)   # before the overfit onset
