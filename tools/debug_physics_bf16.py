"""Per-parameter bf16-vs-fp32 gradient agreement of one full-batch step at the
coauthor-physics production shape (diagnostic for tests/test_gpu_physics_fullsize.py)."""
import os
import sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "linkless-link-prediction_amd"))
import torch  # noqa: E402
import test_gpu_physics_fullsize as T  # noqa: E402

phys = T.physics.__wrapped__() if hasattr(T.physics, "__wrapped__") else None
if phys is None:
    import tempfile
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import llp_split
    import physics_bench
    split = llp_split.production_split("coauthor-physics", os.path.join(tempfile.gettempdir(), "llp_physics"), True)
    phys = (split[0], physics_bench.physics_args())
f32 = T._step(phys, "fp32")
b16 = T._step(phys, "bf16")
print("terms f32", f32.terms[:6].tolist())
print("terms b16", b16.terms[:6].tolist())
for i, (a, b) in enumerate(zip(b16.grads, f32.grads)):
    cos = torch.nn.functional.cosine_similarity(a.flatten().double(), b.flatten().double(), dim=0).item()
    rel = ((a - b).norm() / b.norm()).item()
    print(i, tuple(a.shape), f"cos {cos:.4f} relL2 {rel:.3e} |g|max {b.abs().max().item():.3e} |g| {b.norm().item():.3e}")
