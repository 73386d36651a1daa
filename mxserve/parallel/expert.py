"""Expert parallelism with all-to-all token dispatch (BASELINE.json config 5,
"Mixtral 8x7B ... MoE grouped GEMM + expert all-to-all on 8x MI355X").

The default EP mode of `TransformerLM` ("allreduce") runs every rank's local experts over the
whole replicated batch and sums the partial outputs with the TP all-reduce.  This module is the
all-to-all mode ("a2a"): the replicated hidden states are split into N token slices, each rank
routes ITS slice only, ships every (token, top-k slot) pair to the rank that owns the expert,
runs its local experts over exactly the rows it received (grouped MFMA GEMM, ops.moe_experts),
ships the results back, applies the routing weights and all-gathers the slices so the next
attention layer sees the full batch again.  Per rank and layer the wire traffic is
k*T/N*H (dispatch) + k*T/N*H (combine) + (N-1)/N*T*H (gather) instead of the ring all-reduce's
2(N-1)/N*T*H, and no rank computes routing or experts for tokens it does not own.

Three dispatch layouts:
  ipc       with the custom all-reduce's IPC slots mapped (default for EP <= 8): routing, the
            per-destination stable slot assignment, the row gather and the weighted combine are HIP
            kernels (csrc/kernels/ep.hip, K17 moe_combine) and the all-to-alls push only each
            destination's real rows (counts stay on the device: no host sync, no N x over-send,
            hipGraph-capturable); the slices are all-gathered through the same slots.  A slice
            whose worst-case segment exceeds a slot (prefill chunks: Mixtral at EP = 8 above 4,096
            tokens) runs as several slot-sized chunks, still without a host sync;
  fixed     every destination gets a capacity of C = k * ceil(T/N) rows (the worst case), so all
            splits are equal, nothing is read back to the host and the step stays
            hipGraph-capturable -- decode batches;
  variable  exact per-destination counts exchanged first (one small all-to-all + host read), rows
            sorted by destination -- large prefill chunks, where padding to the worst case would
            ship N x the needed bytes.
RCCL's all_to_all_single over xGMI is one send per peer link, so all 7 links carry a slice at
once -- the collective shape point-to-point xGMI likes, unlike a ring.  With the IPC slots of the
custom all-reduce mapped (MXS_CUSTOM_AR=1), the equal-split exchanges of the fixed layout skip
RCCL: each rank pushes its segments straight into the peers' receive slots (one kernel, all links,
no host involvement; csrc/kernels/custom_allreduce.hip ipc_all_to_all_kernel).
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn.functional as F

from .. import ops

# dispatch pairs per rank above which the exact (host-synchronising) layout is used
FIXED_MAX_PAIRS = 512


def _a2a(out: torch.Tensor, inp: torch.Tensor, group, out_splits=None, in_splits=None) -> torch.Tensor:
    if out_splits is None and inp.is_cuda:
        from .comm import get_tp
        tp = get_tp()
        car = tp.custom_ar
        if car is not None and (group is None or group is tp.group) and car.can_all_to_all(inp):
            return car.all_to_all(out, inp)
    dist.all_to_all_single(out, inp, output_split_sizes=out_splits, input_split_sizes=in_splits, group=group)
    return out


def _ipc_a2a(group, h: torch.Tensor):
    """The custom all-reduce (its IPC slots carry the EP all-to-alls) when it serves this group."""
    if not h.is_cuda:
        return None
    from .comm import get_tp
    tp = get_tp()
    car = tp.custom_ar
    if car is None or car.disabled or not (group is None or group is tp.group):
        return None
    return car


def _gather_slices(out_s: torch.Tensor, T: int, n: int, group) -> torch.Tensor:
    if n == 1:
        return out_s[:T]
    if out_s.is_cuda:
        from .comm import get_tp, tp_all_gather
        tp = get_tp()
        if tp.custom_ar is not None and (group is None or group is tp.group):
            rep = n * out_s.numel() * out_s.element_size()
            if rep // n <= tp.custom_ar.max_bytes and not tp.custom_ar.disabled:
                return tp_all_gather(out_s, dim=0)[:T]
    if out_s.is_cuda and dist.get_backend(group) != "gloo":
        full = torch.empty(n * out_s.shape[0], out_s.shape[1], dtype=out_s.dtype, device=out_s.device)
        dist.all_gather_into_tensor(full, out_s.contiguous(), group=group)
    else:  # gloo (CPU runs, and GPU ranks sharing one device in tests)
        parts = [torch.empty_like(out_s) for _ in range(n)]
        dist.all_gather(parts, out_s.contiguous(), group=group)
        full = torch.cat(parts)
    return full[:T]


def _ipc_chunk(out_c: torch.Tensor, hs: torch.Tensor, tw: torch.Tensor, tid: torch.Tensor, valid: int,
               w13: torch.Tensor, w2: torch.Tensor, top_k: int, n: int, car) -> None:
    """One chunk of a rank's token slice through the IPC dispatch: route (per-destination stable
    slots, csrc/kernels/ep.hip), gather rows, push each destination's real rows into its slot, run
    the local experts over what arrived, push the results back, weighted-combine into out_c."""
    ext = ops.ext()
    dev, H = hs.device, hs.shape[1]
    e_local = w13.shape[0]
    C = hs.shape[0] * top_k  # segment capacity: every pair of the chunk to one destination
    P = C
    tid32 = tid.to(torch.int32).contiguous()
    slot = torch.empty(P, dtype=torch.int32, device=dev)
    send_e = torch.empty(n * C, dtype=torch.int32, device=dev)
    counts = torch.empty(n, dtype=torch.int32, device=dev)
    ext.ep_route(slot, send_e, counts, tid32, valid, e_local, n, C)
    send_x = torch.empty(n * C, H, dtype=hs.dtype, device=dev)  # rows past a segment's count unused
    ext.ep_gather_rows(send_x, hs, slot, top_k)
    recv_e = torch.empty_like(send_e)
    recv_x = torch.empty_like(send_x)
    if n > 1:
        car.all_to_all(recv_e, send_e)  # the ids travel whole (-1 past each count): tiny
        car.all_to_all(recv_x, send_x, counts, H * hs.element_size())
    else:
        recv_e, recv_x = send_e, send_x
    ones = torch.ones(n * C, 1, dtype=torch.float32, device=dev)
    y = ops.moe_experts(recv_x, w13, w2, ones, recv_e.unsqueeze(1), 0)
    rcounts = torch.empty(n, dtype=torch.int32, device=dev)
    ext.ep_segment_rows(rcounts, recv_e, C)
    back = y
    if n > 1:
        back = torch.empty_like(y)
        car.all_to_all(back, y, rcounts, H * hs.element_size())
    ext.moe_combine(out_c, back, tw.float().contiguous(), slot)  # K17: weighted gather, fp32 accumulate


def moe_a2a(h: torch.Tensor, gate_w: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor, top_k: int,
            rank: int, world: int, group=None, force_layout: str | None = None) -> torch.Tensor:
    """h [T, H] replicated on every rank -> MoE output [T, H] replicated on every rank.
    gate_w [E, H] (replicated router), w13 [E_local, 2I, H], w2 [E_local, H, I] (this rank's
    experts, global ids rank*E_local ...)."""
    T, H = h.shape
    e_local = w13.shape[0]
    n = world
    S = (T + n - 1) // n  # token slice per rank (padded)
    lo = min(T, rank * S)
    hi = min(T, lo + S)
    dev = h.device
    hs = torch.zeros(S, H, dtype=h.dtype, device=dev)
    hs[:hi - lo] = h[lo:hi]
    row_ok = torch.arange(S, device=dev) < (hi - lo)
    tw, tid = ops.moe_topk_softmax(F.linear(hs, gate_w), top_k)  # [S, k]
    P = S * top_k
    dest = (tid.long() // e_local).reshape(P)
    pair_ok = row_ok.repeat_interleave(top_k)
    local_eid = (tid.long().reshape(P) - dest * e_local).to(torch.int32)
    tok = torch.arange(P, device=dev) // top_k
    car = _ipc_a2a(group, h)
    if force_layout is not None:
        layout = force_layout
    elif n > 1 and car is not None and top_k * H * h.element_size() <= car.max_bytes:
        layout = "ipc"  # device-side dispatch, in slot-sized chunks of the slice
    else:
        layout = "fixed" if P <= FIXED_MAX_PAIRS else "variable"

    if layout == "ipc":
        # one destination segment of a chunk (k x rows pairs) must fit an IPC slot: a prefill slice
        # larger than that runs as several chunks, every one on the device (no host sync), the same
        # number on every rank (S is equal everywhere)
        sc = S if force_layout == "ipc" and n == 1 else max(1, car.max_bytes // (top_k * H * h.element_size()))
        out_s = torch.empty(S, H, dtype=h.dtype, device=dev)
        valid = hi - lo
        for c0 in range(0, S, sc):
            c1 = min(S, c0 + sc)
            _ipc_chunk(out_s[c0:c1], hs[c0:c1], tw[c0:c1], tid[c0:c1], max(0, min(valid - c0, c1 - c0)),
                       w13, w2, top_k, n, car)
        return _gather_slices(out_s, T, n, group)

    if layout == "fixed":
        C = P
        # slot of each pair inside its destination's segment: running count of earlier pairs with
        # the same destination (one-hot prefix sum, P x N elements)
        onehot = F.one_hot(dest.clamp(0, n - 1), n) * pair_ok.unsqueeze(1)
        pos = (onehot.cumsum(0) - 1).gather(1, dest.clamp(0, n - 1).unsqueeze(1)).squeeze(1)
        idx = torch.where(pair_ok, dest * C + pos, torch.full_like(dest, n * C))  # invalid -> spill row
        send_x = torch.zeros(n * C + 1, H, dtype=h.dtype, device=dev)
        send_x.index_copy_(0, idx, hs.index_select(0, tok))
        send_e = torch.full((n * C + 1,), -1, dtype=torch.int32, device=dev)
        send_e.index_copy_(0, idx, local_eid)
        recv_x = torch.empty(n * C, H, dtype=h.dtype, device=dev)
        recv_e = torch.empty(n * C, dtype=torch.int32, device=dev)
        if n > 1:
            _a2a(recv_x, send_x[:n * C], group)
            _a2a(recv_e, send_e[:n * C], group)
        else:
            recv_x.copy_(send_x[:C])
            recv_e.copy_(send_e[:C])
        ones = torch.ones(n * C, 1, dtype=torch.float32, device=dev)
        y = ops.moe_experts(recv_x, w13, w2, ones, recv_e.unsqueeze(1), 0)
        back = torch.empty_like(y)
        if n > 1:
            _a2a(back, y, group)
        else:
            back.copy_(y)
        back = torch.cat([back, torch.zeros(1, H, dtype=back.dtype, device=dev)])
        yp = back.index_select(0, idx)  # [P, H], invalid pairs read the zero row
    else:
        key = torch.where(pair_ok, dest, torch.full_like(dest, n))  # invalid pairs sort last
        order = torch.sort(key, stable=True).indices
        counts = torch.bincount(key, minlength=n + 1)[:n]
        nsend = int(counts.sum())
        order = order[:nsend]
        if n > 1:
            rc = torch.empty_like(counts)
            _a2a(rc, counts, group)
            send_splits, recv_splits = counts.tolist(), rc.tolist()
        else:
            send_splits = recv_splits = [nsend]
        nrecv = sum(recv_splits)
        send_x = hs.index_select(0, tok.index_select(0, order))
        send_e = local_eid.index_select(0, order).contiguous()
        recv_x = torch.empty(nrecv, H, dtype=h.dtype, device=dev)
        recv_e = torch.empty(nrecv, dtype=torch.int32, device=dev)
        if n > 1:
            _a2a(recv_x, send_x, group, recv_splits, send_splits)
            _a2a(recv_e, send_e, group, recv_splits, send_splits)
        else:
            recv_x.copy_(send_x)
            recv_e.copy_(send_e)
        ones = torch.ones(nrecv, 1, dtype=torch.float32, device=dev)
        y = ops.moe_experts(recv_x, w13, w2, ones, recv_e.unsqueeze(1), 0) if nrecv else recv_x
        back = torch.empty(nsend, H, dtype=h.dtype, device=dev)
        if n > 1:
            _a2a(back, y, group, send_splits, recv_splits)
        else:
            back.copy_(y)
        yp = torch.zeros(P, H, dtype=h.dtype, device=dev)
        yp.index_copy_(0, order, back)

    # combine: out[t] = sum_j w[t, j] * y[t, j]  (fp32 accumulate)
    out_s = (yp.float().reshape(S, top_k, H) * tw.float().unsqueeze(2)).sum(1).to(h.dtype)
    return _gather_slices(out_s, T, n, group)
