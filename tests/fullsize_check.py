"""Shared checker of the full-size oracle tests (test_gpu_fullsize_oracle.py: collab minibatch,
BASELINE configs[2]; test_gpu_physics_fullsize.py: coauthor-physics full batch, configs[3]).

One HIP engine step is compared with the CPU oracle (oracle/llp_oracle.py) run on the same
injected draws twice: in float64 (the truth) and in float32 (the reference's own arithmetic,
torch on the CPU).  Bars:
  (1) logits (north_star "within 1e-4 on logits"): s_r, t_r, out -- the reference's sigmoid
      outputs (src/main.py:105-106,126 / 186-187,213) -- within 1e-4 of the f64 oracle's, and the
      student's pre-sigmoid logits within 1e-4 * max(1, |z|);
  (2) every loss term within 1e-4 * max(1, |term|);
  (3) every gradient (after clip_grad_norm_, which scales .grad in place in both) within 2e-4
      of its largest magnitude of the f64 oracle, or within 4x the
      error of the reference's fp32 arithmetic where that is larger (a weight gradient here is a
      cancelling sum over 10^5 - 10^6 rows, whose fp32 rounding is inherent to the arithmetic);
  (4) after clip + Adam (src/main.py:132-138) every parameter whose clipped gradient is large
      enough that Adam's update lr * g / (|g| + eps) is insensitive to the gradient's rounding
      (check() states the threshold) within 1e-4 * lr of the f64 oracle's, and every parameter
      within 2 lr.
Test infrastructure only (the oracle is the checker)."""
import numpy as np
import torch


def oracle_step(O, losses, params0, L, lr, d):
    """The oracle's loss dict + clip + Adam in dtype ``d``.  ``losses(leaves_stu_w, stu_b, pred_w,
    pred_b, d)`` returns distill_losses_*'s dict.  Returns (terms + logits, clipped grads, new
    params, clip coefficient per param)."""
    leaves = [p.to(d).clone().requires_grad_() for p in params0]
    sw, sb = leaves[0:2 * L:2], leaves[1:2 * L:2]
    pw, pb = leaves[2 * L::2], leaves[2 * L + 1::2]
    prev = torch.get_default_dtype()
    torch.set_default_dtype(d)          # the oracle's label vector (torch.ones / zeros) in d too
    try:
        r = losses(sw, sb, pw, pb, d)
        adam = O.AdamState(leaves, lr=lr)
        new, grads_clip, norms = O.distill_step(leaves[:2 * L], leaves[2 * L:], adam, r["loss"])
    finally:
        torch.set_default_dtype(prev)
    # clip_grad_norm_ (max_norm 1, src/main.py:134-135) scales .grad in place, in the reference and
    # in the engine's clip + Adam launch: after the step both hold the CLIPPED gradient
    coefs = []
    for grp, total in ((slice(0, 2 * L), norms[0]), (slice(2 * L, len(params0)), norms[1])):
        coefs += [min(1.0, 1.0 / (float(total) + 1e-6))] * len(grads_clip[grp])
    terms = {k: r[k].item() for k in ("loss", "label_loss", "llp_d", "llp_r")}
    terms["logits"] = {k: r[k].detach().double() for k in ("s_r", "t_r", "out")}
    return terms, [gc.detach() for gc in grads_clip], [p.detach() for p in new], coefs


def check(lg, terms, grads_gpu, params1, params0, o64, o32, lr, shape_ctx, n_lab, min_live=0.5, z_max=15.0,
          need_clip=True):
    """Assert bars (1)-(4) (module docstring).  lg: engine.last_logits() on the host (double);
    terms: engine.terms; grads_gpu: the engine's .grad after the step (clipped, as the reference's);
    o64 / o32: oracle_step's results in float64 / float32.  need_clip: the state must put both
    clip coefficients below 1."""
    t64, g64, p64, coef64 = o64
    _, g32, _, _ = o32
    # (1) logits
    ref = t64["logits"]
    assert lg["s_r"].shape == ref["s_r"].shape == shape_ctx, (lg["s_r"].shape, ref["s_r"].shape)
    assert lg["out"].shape == ref["out"].shape == (n_lab,), (lg["out"].shape, ref["out"].shape)
    print("logits: max |HIP - f64 oracle|  s_r %.2e  t_r %.2e  out %.2e" % tuple(
        (lg[k] - ref[k]).abs().max().item() for k in ("s_r", "t_r", "out")), flush=True)
    for k in ("s_r", "t_r", "out"):
        assert (lg[k] - ref[k]).abs().max().item() <= 1e-4, k
    for k, zk in (("s_r", "s_logit"), ("out", "out_logit")):
        p_ref = ref[k].clamp(1e-300, 1 - 1e-16)
        z_ref = torch.log(p_ref) - torch.log1p(-p_ref)
        err = ((lg[zk] - z_ref).abs() / z_ref.abs().clamp(min=1.0)).max().item()
        print(f"  {zk}: |z| max {z_ref.abs().max().item():.2f}, max error / max(1, |z|) {err:.2e}", flush=True)
        assert err <= 1e-4, (zk, err)
    # the state keeps the label logits' f32 sigmoids unsaturated: BCE's log(1 - o) of an o that
    # rounds to 1.0 in f32 (z > ~16.6) is clamped to -100 by nn.BCELoss, where f64 gives -z, so
    # the fp32 arithmetic (the reference's and this one) would leave the f64 truth by design
    p_out = ref["out"].clamp(1e-300, 1 - 1e-16)
    z_out = (torch.log(p_out) - torch.log1p(-p_out)).abs().max().item()
    assert z_out < z_max, z_out
    # the state the callers describe: logits spread (and both clip coefficients below 1)
    assert ref["s_r"].max().item() > 0.9 and ref["s_r"].min().item() < 0.1
    if need_clip:
        assert max(coef64) < 1.0, coef64
    # (2) loss terms
    for i, k in ((0, "loss"), (1, "label_loss"), (2, "llp_d"), (3, "llp_r")):
        r = t64[k]
        print(f"  {k}: HIP {terms[i].item():.7f}  f64 oracle {r:.7f}", flush=True)
        assert abs(terms[i].item() - r) <= 1e-4 * max(1.0, abs(r)), (k, terms[i].item(), r)
    # (3) gradients
    rows_err = []
    for a, b, c, p in zip(grads_gpu, g64, g32, params0):
        m = b.abs().max().item()
        e_hip = (a.double() - b).abs().max().item()
        e_ref = (c.double() - b).abs().max().item()
        rows_err.append((tuple(p.shape), m, e_hip, e_ref))
    print("gradient max |g|, then error / max |g| (HIP fp32 | reference fp32) per tensor:", flush=True)
    for shape, m, e_hip, e_ref in rows_err:
        print(f"  {str(shape):14s} {m:.3e}  {e_hip / m:.2e} | {e_ref / m:.2e}", flush=True)
    for shape, m, e_hip, e_ref in rows_err:
        assert e_hip <= max(2e-4 * m, 4.0 * e_ref), (shape, m, e_hip, e_ref)
    # (4) parameters after clip + Adam.  Adam's first update lr * g / (|g| + eps) moves by
    # lr * eps * dg / g^2 for a gradient error dg: an entry is "live" (its update insensitive to
    # the gradient's rounding, within 1e-4 lr / 4) where |g| >= max(1e-5, 2 sqrt(eps dg / 1e-4)),
    # dg = the HIP tensor's measured max error (eps = 1e-8)
    n_live = n_all = 0
    for a, b, gref, (_, _, e_hip, _) in zip(params1, p64, g64, rows_err):
        d = (a.double() - b).abs()
        assert d.max().item() <= 2 * lr * (1 + 1e-3), d.max().item()
        live = gref.abs() >= max(1e-5, 2.0 * (1e-8 * e_hip / 1e-4) ** 0.5)   # (gref: the clipped gradient)
        n_live += int(live.sum())
        n_all += live.numel()
        if bool(live.any()):
            assert d[live].max().item() <= 1e-4 * lr + 1e-8, d[live].max().item()
    print(f"post-Adam check: {n_live} of {n_all} parameters live ({n_live / n_all:.1%}); clip coefficients "
          f"{sorted(set(round(c, 4) for c in coef64))}", flush=True)
    assert n_live >= min_live * n_all
    assert np.isfinite(terms.numpy()).all()
