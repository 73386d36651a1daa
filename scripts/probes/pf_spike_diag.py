"""Which outputs of the v3 softmax variants miss the fp32 reference on the x12 spike case."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from mxserve import ops  # noqa: E402
from mxserve.ops import reference as ref  # noqa: E402
from test_kernels_gpu import _paged_setup  # noqa: E402

torch.manual_seed(0)
gpu = "cuda:0"
D, G, hkv = 64, 4, 1
kv, bt = _paged_setup([256], hkv, D, device=gpu)
q = torch.randn(256, G, D, device=gpu, dtype=torch.bfloat16)
for key, (tok, head) in ((200, (255, 0)), (130, (140, 2)), (161, (200, 1)), (230, (255, 0))):
    kv[int(bt[0, key // 16]), 1, 0, 0, key % 16, :] = q[tok, head] * 12
qsl = torch.tensor([0, 256], dtype=torch.int32)
sl = torch.tensor([256], dtype=torch.int32)
exp = ref.paged_attention(q.cpu(), kv[:, 1].cpu(), bt, qsl, sl, 0.125).float()
for var in (0, 1, 2, 3, 7):
    out = ops.paged_attention_prefill(q, kv[:, 1], bt.to(gpu), qsl.to(gpu), sl.to(gpu), 0.125, 256,
                                      version=0x100 | var).float().cpu()
    err = (out - exp).abs()
    bad = (err > 0.03 + 0.03 * exp.abs()).nonzero().tolist()
    print("var", var, "max err", round(err.max().item(), 4), "bad", len(bad), bad[:6],
          [(round(out[t, h, d].item(), 4), round(exp[t, h, d].item(), 4)) for t, h, d in bad[:6]], flush=True)
    rows = err.amax(-1)
    top = torch.topk(rows.flatten(), 5)
    print("   worst rows (tok, head, err):", [(i // G, i % G, round(v, 4)) for v, i in zip(top.values.tolist(), top.indices.tolist())])
