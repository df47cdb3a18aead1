import sys, os
R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
for p in ("tests", "", "linkless-link-prediction_amd"):
    sys.path.insert(0, os.path.join(R, p))
import torch
import golden_io as G
import test_gpu_teacher as T
from oracle import llp_oracle as O
c = G.load_teacher_case("teacher_sage_small")
eng, model, pred = T._build(c)
pairs = c.pos_train_edge.to(torch.int32).to("cuda").contiguous()
st = c.steps[0]
eng.step(st.link_perm.to(torch.int32).to("cuda"), pairs, neg=st.neg_edge.to("cuda"))
torch.cuda.synchronize()
convs = [tuple(c.enc0[3 * i:3 * i + 3]) for i in range(c.L)]
h = O.sage_forward(c.x, c.edge_index, convs, 0.0, updated=False)
print("h diff", (eng.h.cpu() - h).abs().max().item(), h.abs().max().item())
tr = torch.cat([st.edge, st.neg_edge], 1)
_, lg = O.link_predictor_forward(h[tr[0]], h[tr[1]], c.pred0[0::2], c.pred0[1::2], return_logit=True)
R_ = tr.shape[1]
print("R", R_, "P", st.edge.shape[1], "neg", st.neg_edge.shape)
got = eng._bufs["logit"][:R_].cpu()
print("logit diff", (got - lg.squeeze(-1)).abs().max().item())
ia = eng._bufs["t_ia"][:R_].cpu(); ib = eng._bufs["t_ib"][:R_].cpu()
print("ia ok", bool((ia == tr[0]).all()), "ib ok", bool((ib == tr[1]).all()))
bad = (ia != tr[0]).nonzero().flatten()[:10]
print("bad idx", bad.tolist(), ia[bad].tolist(), tr[0][bad].tolist())
print("pairs shape", c.pos_train_edge.shape, "perm max", st.link_perm.max().item())
import torch.nn.functional as F
L0, L1 = eng.layers
src, dst = c.edge_index[0], c.edge_index[1]
agg0 = O.sage_mean_aggregate(c.x, src, dst, c.N)
print("XA0 right vs x", (L0["XA"][:, 24:].cpu() - c.x).abs().max().item())
print("XA0 left vs agg", (L0["XA"][:, :24].cpu() - agg0).abs().max().item())
y0 = F.relu(F.linear(agg0, c.enc0[0], c.enc0[1]) + F.linear(c.x, c.enc0[2]))
print("X1 vs relu(conv0)", (L1["XA"][:, 64:].cpu() - y0).abs().max().item())
agg1 = O.sage_mean_aggregate(y0, src, dst, c.N)
print("XA1 left vs agg1", (L1["XA"][:, :64].cpu() - agg1).abs().max().item())
Wc = L0["Wf"].cpu()
print("Wcat0 ok", (Wc[:, :24] - c.enc0[0]).abs().max().item(), (Wc[:, 24:] - c.enc0[2]).abs().max().item())
Wc1 = L1["Wf"].cpu()
print("Wcat1 ok", (Wc1[:, :64] - c.enc0[3]).abs().max().item(), (Wc1[:, 64:] - c.enc0[5]).abs().max().item())
