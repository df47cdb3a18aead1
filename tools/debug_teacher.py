import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "linkless-link-prediction_amd"))
import torch
import golden_io as G
import test_gpu_teacher as T
for name in G.TEACHER_CASES:
    c = G.load_teacher_case(name)
    eng, model, pred = T._build(c)
    pairs = c.pos_train_edge.to(torch.int32).to("cuda").contiguous()
    st = c.steps[0]
    eng.step(st.link_perm.to(torch.int32).to("cuda"), pairs, neg=st.neg_edge.to("cuda"))
    torch.cuda.synchronize()
    names = [n for n, _ in model.named_parameters()] + [n for n, _ in pred.named_parameters()]
    for n, p, ref in zip(names, list(model.parameters()) + list(pred.parameters()), st.grads):
        g = p.grad.detach().cpu()
        print(name, n, tuple(p.shape), "err %.3e ref %.3e" % ((g - ref).abs().max().item(), ref.abs().max().item()),
              "ratio-fit %.4f" % ((g * ref).sum() / (ref * ref).sum()).item())
