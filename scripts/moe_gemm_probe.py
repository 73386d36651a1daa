"""Mixtral-8x7B expert GEMMs alone (decode-sized routed rows): gate_up (SiLU epilogue) and down
grouped MFMA GEMMs, time and effective weight bandwidth."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch  # noqa: E402

from mxserve import ops  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    dev = torch.device("cuda:0")
    H, I, E, K = 4096, 14336, 8, 2
    w13 = torch.randn(E, 2 * I, H, device=dev, dtype=torch.bfloat16) * 0.02
    w2 = torch.randn(E, H, I, device=dev, dtype=torch.bfloat16) * 0.02
    for T in (16, 64, 256):
        ids = torch.stack([torch.randperm(E, device=dev)[:K] for _ in range(T)]).to(torch.int32)
        offs = torch.empty(E + 1, dtype=torch.int32, device=dev)
        perm = torch.full((T * K,), -1, dtype=torch.int32, device=dev)
        ops.ext().moe_align(offs, perm, ids, 0, E)
        xs = torch.randn(T * K, H, device=dev, dtype=torch.bfloat16)
        h = torch.empty(T * K, I, device=dev, dtype=torch.bfloat16)
        ys = torch.empty(T * K, H, device=dev, dtype=torch.bfloat16)
        t13 = timeit(lambda: ops.ext().moe_grouped_gemm(h, xs, w13, offs, True))
        t2 = timeit(lambda: ops.ext().moe_grouped_gemm(ys, h, w2, offs, False))
        part = torch.empty(8, T * K, H, device=dev, dtype=torch.float32)
        t2s = {sp: timeit(lambda: ops.ext().moe_grouped_gemm(ys, h, w2, offs, False, sp, part)) for sp in (2, 4, 8)}
        n_act = int((torch.bincount(ids.flatten().long(), minlength=E) > 0).sum())
        print(json.dumps({"T": T, "experts_active": n_act, "gate_up_ms": round(t13, 4), "down_ms": round(t2, 4),
                          "gate_up_TBps": round(n_act * 2 * I * H * 2 / t13 / 1e9, 2),
                          "down_TBps": round(n_act * H * I * 2 / t2 / 1e9, 2),
                          **{f"down_split{sp}_ms": round(v, 4) for sp, v in t2s.items()}}), flush=True)
        # one local expert (EP = 8): rows of expert 0 only
        offs1 = torch.tensor([0, T * K // 4], dtype=torch.int32, device=dev)
        t1 = {sp: timeit(lambda: ops.ext().moe_grouped_gemm(ys, h, w2[:1].contiguous(), offs1, False, sp, part))
              for sp in (1, 4, 8)}
        w1 = w13[:1].contiguous()
        x1 = torch.randn(T * K // 4, H, device=dev, dtype=torch.bfloat16)
        h1 = torch.empty(T * K // 4, I, device=dev, dtype=torch.bfloat16)
        p13 = torch.empty(4, T * K // 4, 2 * I, device=dev, dtype=torch.float32)

        def gu_split():
            ops.ext().moe_grouped_gemm(h1.new_empty(0, 2 * I), x1, w1, offs1, False, 4, p13)
            ops.ext().silu_mul_partials(h1, p13)
        t1["gate_up_silu"] = timeit(lambda: ops.ext().moe_grouped_gemm(h1, x1, w1, offs1, True))
        t1["gate_up_split4_then_silu"] = timeit(gu_split)
        print(json.dumps({"T": T, "ep8_one_expert_rows": T * K // 4,
                          **{(f"down_split{sp}_ms" if isinstance(sp, int) else f"{sp}_ms"): round(v, 4)
                             for sp, v in t1.items()}}), flush=True)


if __name__ == "__main__":
    main()
