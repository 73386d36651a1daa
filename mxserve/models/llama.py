"""Decoder-only transformer for the Llama / Qwen3 / Mixtral families over a paged KV cache.

One forward = one engine step over a flattened token batch (decode tokens first, then prefill
chunks; SURVEY.md §3.3 kernel sequence K01 -> L x [K02, K05, K04, K11|K12, K06, K02, K07, K10, K08]
-> K02 -> K09).  Tensor parallelism: fused QKV / gate-up projections are
column-parallel (whole heads per rank), o/down projections row-parallel followed by one all-reduce
each, the LM head is vocab-parallel (all-gather of fp32 logits).  Mixtral MLPs are replaced by a
top-2 MoE block whose experts are sharded over the same ranks (expert parallel, §2.4 P06).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn.functional as F

from .. import ops
from ..ops import reference as ref
from ..parallel.comm import get_tp, tp_add_rms_norm, tp_all_gather, tp_all_reduce, tp_linear_add_rms_norm
from .config import ModelConfig


@dataclass
class AttnMetadata:
    """Per-step batch description (host ints + device tensors)."""
    positions: torch.Tensor  # [T] int64
    slot_mapping: torch.Tensor  # [T] int64
    block_tables: torch.Tensor  # [S, max_blocks] int32
    seq_lens: torch.Tensor  # [S] int32 total tokens in cache after this step
    query_start_loc: torch.Tensor  # [S+1] int32
    logits_indices: torch.Tensor  # [S_sample] int64 rows of hidden to project
    num_decodes: int  # first num_decodes sequences have exactly one query token
    num_prefills: int
    num_prefill_tokens: int
    max_query_len: int
    max_seq_len: int
    prefill_query_start_loc: Optional[torch.Tensor] = None  # [P+1] int32, rebased at 0
    sample_seq: Optional[torch.Tensor] = None  # [S_sample] int32: sequence of each logits row

    @property
    def num_tokens(self) -> int:
        return self.num_decodes + self.num_prefill_tokens


def _shard_rows(w: torch.Tensor, rank: int, size: int) -> torch.Tensor:
    n = w.shape[0] // size
    return w[rank * n:(rank + 1) * n]


def _shard_cols(w: torch.Tensor, rank: int, size: int) -> torch.Tensor:
    n = w.shape[1] // size
    return w[:, rank * n:(rank + 1) * n]


class TransformerLM:
    """Weights live in a flat dict of tensors (no nn.Module overhead on the hot path)."""

    def __init__(self, cfg: ModelConfig, device: torch.device, dtype: torch.dtype = torch.bfloat16,
                 moe_dispatch: str = "allreduce"):
        if moe_dispatch not in ("allreduce", "a2a"):
            raise ValueError(f"moe_dispatch must be allreduce|a2a, got {moe_dispatch!r}")
        self.cfg = cfg
        self.moe_dispatch = moe_dispatch
        # last layer of a prefill step: attention/o_proj/MLP only for the rows that produce logits
        self.prune_last_layer = os.environ.get("MXS_PRUNE_LAST_LAYER", "1") == "1"
        # TP = 1 on the GPU: o_proj / down_proj end in the next RMSNorm (ops.linear_add_rms_norm: a
        # split-K projection's slabs go straight into one sum + residual add + norm kernel)
        self.fuse_residual = os.environ.get("MXS_FUSE_RESIDUAL", "1") == "1"
        # TP = 1 dense models on the GPU, prefill / mixed steps: RMSNorms inside the consumer GEMMs and
        # residual adds inside the producers (_forward_pf); self.wf holds the norm-folded weights
        self.fuse_prefill = os.environ.get("MXS_PF_FUSED", "1") == "1"
        # pure-decode steps of more than 256 rows: the prefill chain (_forward_pf: gemm_pf / the
        # prefill-bucket tables) or the decode chain (_forward_fused: the decode table's tuned forms
        # with their rope / add+norm epilogues).  MXS_PF_DECODE=1 keeps the prefill chain.
        self.pf_decode = os.environ.get("MXS_PF_DECODE", "1") == "1"
        self.pf_chain = False
        self.wf: dict[str, torch.Tensor] = {}
        # fp8 KV cache: stored = x / scale, per layer (1.0 until the runner calibrates them from a
        # probe prefill, mxserve/engine/model_runner.py::_calibrate_kv_scales; MXS_KV_SCALE fixes all)
        ks = float(os.environ.get("MXS_KV_SCALE", "1.0"))
        self.kv_scales = [{"k_scale": ks, "v_scale": ks} for _ in range(cfg.num_layers)]
        self.device = torch.device(device)
        self.dtype = dtype
        tp = get_tp()
        self.tp_rank, self.tp_size = tp.tp_rank, tp.tp_size
        if cfg.num_heads % self.tp_size:
            raise ValueError("num_heads must divide by tp_size")
        self.nh = cfg.num_heads // self.tp_size
        # KV heads: split when possible, otherwise replicate (e.g. 8 kv heads over tp=16)
        self.kv_replicas = max(1, self.tp_size // cfg.num_kv_heads)
        self.nkv = max(1, cfg.num_kv_heads // self.tp_size)
        self.hd = cfg.head_dim
        self.scale = 1.0 / math.sqrt(self.hd)
        self.w: dict[str, torch.Tensor] = {}
        self.cos_sin = ref.build_cos_sin_cache(cfg.head_dim, cfg.max_position_embeddings, cfg.rope_theta,
                                               cfg.rope_scaling, device=self.device)
        if cfg.is_moe:
            if cfg.num_experts % self.tp_size:
                raise ValueError("num_experts must divide by tp_size for expert parallelism")
            self.e_local = cfg.num_experts // self.tp_size
            self.e_offset = self.tp_rank * self.e_local
        self.vocab_local = (cfg.vocab_size + self.tp_size - 1) // self.tp_size

    # ------------------------------------------------------------------ weights
    def local_shapes(self) -> dict[str, tuple]:
        c = self.cfg
        H, D = c.hidden_size, c.head_dim
        shapes = {"embed": (c.vocab_size, H), "norm": (H,)}
        if not c.tie_word_embeddings:
            shapes["lm_head"] = (self.vocab_local, H)
        I_loc = c.intermediate_size // self.tp_size if not c.is_moe else c.intermediate_size
        for i in range(c.num_layers):
            p = f"l{i}."
            shapes[p + "in_norm"] = (H,)
            shapes[p + "post_norm"] = (H,)
            shapes[p + "qkv"] = ((self.nh + 2 * self.nkv) * D, H)
            shapes[p + "o"] = (H, self.nh * D)
            if c.qk_norm:
                shapes[p + "q_norm"] = (D,)
                shapes[p + "k_norm"] = (D,)
            if c.is_moe:
                shapes[p + "gate"] = (c.num_experts, H)
                shapes[p + "w13"] = (self.e_local, 2 * I_loc, H)
                shapes[p + "w2"] = (self.e_local, H, I_loc)
            else:
                shapes[p + "gate_up"] = (2 * I_loc, H)
                shapes[p + "down"] = (H, I_loc)
        return shapes

    def init_random(self, seed: int = 0, std: float = 0.02) -> None:
        """Random-init this rank's shard directly on the device (no host staging).  Synthetic
        weights per the north star: no checkpoints are reachable on the GPU box."""
        g = torch.Generator(device=self.device)
        g.manual_seed(seed * 1000003 + self.tp_rank)
        for name, shape in self.local_shapes().items():
            if name.endswith("norm"):
                t = torch.ones(shape, dtype=self.dtype, device=self.device)
            else:
                t = torch.empty(shape, dtype=self.dtype, device=self.device)
                t.normal_(0.0, std, generator=g)
            self.w[name] = t

    def load_full_state(self, full: dict[str, torch.Tensor]) -> None:
        """Take unsharded weights in this module's naming (see weights.py) and keep this rank's
        shard.  Used by the safetensors loader and by TP/EP equivalence tests."""
        c, r, s = self.cfg, self.tp_rank, self.tp_size
        D = c.head_dim
        out = {}
        for name, t in full.items():
            if name == "lm_head":
                t = _pad_rows(t, self.vocab_local * s)
                t = _shard_rows(t, r, s)
            elif name.endswith(".qkv"):
                qs, ks = c.num_heads * D, c.num_kv_heads * D
                q, k, v = t[:qs], t[qs:qs + ks], t[qs + ks:]
                kr = r // self.kv_replicas if self.kv_replicas > 1 else r
                ksz = s // self.kv_replicas if self.kv_replicas > 1 else s
                t = torch.cat([_shard_rows(q, r, s), _shard_rows(k, kr, ksz), _shard_rows(v, kr, ksz)])
            elif name.endswith(".o"):
                t = _shard_cols(t, r, s)
            elif name.endswith(".gate_up"):
                I = c.intermediate_size
                t = torch.cat([_shard_rows(t[:I], r, s), _shard_rows(t[I:], r, s)])
            elif name.endswith(".down"):
                t = _shard_cols(t, r, s)
            elif name.endswith(".w13") or name.endswith(".w2"):
                t = t[self.e_offset:self.e_offset + self.e_local]
            out[name] = t.to(device=self.device, dtype=self.dtype).contiguous()
        if c.tie_word_embeddings:
            out.pop("lm_head", None)
        self.w = out

    def prepare_fused_prefill(self, tuning: bool = True, max_rows: int = 8192) -> bool:
        """Norm-folded copies of the qkv / gate_up weights (W diag(g), ops.fold_norm_weight) for the
        prefill forward whose RMSNorms run inside the consumer GEMMs (_forward_pf).  TP = 1 dense
        models on the GPU.  Call after the weights are final and before the KV pool is sized: the
        copies take the qkv + gate_up bytes of every layer once more (1.3 GB for Llama-3.2-1B), so a
        copy is only made when its row-scaled form can run at all: the start-up tuner will run
        (`tuning`: not enforce_eager) and the stored table does not already reject it at every row
        bucket (ops/prefill_pf.py folded_weight_needed)."""
        from ..ops import prefill_pf
        c = self.cfg
        self.wf = {}
        self.pf_chain = (self.fuse_prefill and self.fuse_residual and self.device.type == "cuda" and
                         self.tp_size == 1 and not c.is_moe and c.hidden_size % 64 == 0)
        if not self.pf_chain or not tuning:
            return False
        want = {name: prefill_pf.folded_weight_needed(*self.w["l0." + name].shape, code, max_rows, self.device)
                for name, code in (("qkv", prefill_pf.CODE_RS), ("gate_up", prefill_pf.CODE_RS_SWIGLU))}
        norms = {"qkv": "in_norm", "gate_up": "post_norm"}
        for i in range(c.num_layers):
            p = f"l{i}."
            for name, keep in want.items():
                if keep:
                    self.wf[p + name] = ops.fold_norm_weight(self.w[p + name], self.w[p + norms[name]])
        return bool(self.wf)

    def drop_folded(self, names) -> None:
        """Free the folded copies of projections (e.g. "qkv", "gate_up") whose row-scaled form the
        start-up tuner rejected at every row bucket: norm_linear then always takes the norm pass."""
        for k in [k for k in self.wf if k.split(".", 1)[1] in set(names)]:
            del self.wf[k]

    def lm_head_weight(self) -> torch.Tensor:
        if self.cfg.tie_word_embeddings:
            if self.tp_size == 1:
                return self.w["embed"]
            if "_lm_head_tied" not in self.w:
                e = _pad_rows(self.w["embed"], self.vocab_local * self.tp_size)
                self.w["_lm_head_tied"] = _shard_rows(e, self.tp_rank, self.tp_size).contiguous()
            return self.w["_lm_head_tied"]
        return self.w["lm_head"]

    # ------------------------------------------------------------------ forward
    def _fused_q_rope(self, h: torch.Tensor, i: int, qkv_given: bool = False) -> bool:
        """Prefill / mixed steps on the GPU (hipBLASLt qkv, M > 256): the rope kernel writes only K / V
        and both attention kernels read q from the qkv rows and rotate it while loading it (one
        [T, Hq, D] write + read less per layer).  Needs the MFMA decode kernel (G >= 4) and no q/k
        norm; MXS_FUSED_Q_ROPE=0 turns it off."""
        return (_FUSED_Q_ROPE and h.is_cuda and h.shape[0] > 256 and not self.cfg.qk_norm and
                self.hd in (64, 128) and self.nh // self.nkv >= 4 and self.nh % self.nkv == 0 and
                (qkv_given or not ops.qkv_uses_slabs(h, self.w[f"l{i}.qkv"])))

    def _side_stream(self, device) -> Optional[torch.cuda.Stream]:
        """The mixed-step prefill-attention stream (None while a graph is being captured)."""
        if torch.cuda.is_current_stream_capturing():
            return None
        st = getattr(self, "_attn_side", None)
        if st is None:
            st = self._attn_side = torch.cuda.Stream(device=device)
        return st

    def _attention(self, i: int, h: Optional[torch.Tensor], md: AttnMetadata, kv_layer: torch.Tensor,
                   project: bool = True, qkv: Optional[torch.Tensor] = None):
        """qkv: the projection already computed (_forward_pf); h is then unused."""
        c, w, p = self.cfg, self.w, f"l{i}."
        rope = None
        if self._fused_q_rope(h if qkv is None else qkv, i, qkv is not None):
            if qkv is None:
                qkv = ops.linear(h, w[p + "qkv"])
            q = ops.rope_kv_into_cache(qkv, self.nh, self.nkv, self.hd, md.positions,
                                       self.cos_sin, kv_layer, md.slot_mapping, **self.kv_scales[i],
                                       num_decodes=md.num_decodes)
            rope = (md.positions, self.cos_sin)
        elif qkv is not None:
            q = ops.rope_and_cache(qkv, self.nh, self.nkv, self.hd, md.positions, self.cos_sin, kv_layer,
                                   md.slot_mapping, w.get(p + "q_norm"), w.get(p + "k_norm"), c.rms_norm_eps,
                                   **self.kv_scales[i])
        else:
            q = ops.linear_rope_and_cache(h, w[p + "qkv"], self.nh, self.nkv, self.hd, md.positions, self.cos_sin,
                                          kv_layer, md.slot_mapping, w.get(p + "q_norm"), w.get(p + "k_norm"),
                                          c.rms_norm_eps, **self.kv_scales[i])
        nd = md.num_decodes
        if not q.is_cuda:
            o = ref.paged_attention(q, kv_layer, md.block_tables, md.query_start_loc, md.seq_lens, self.scale,
                                    **self.kv_scales[i])
        elif md.num_prefills == 0:
            o = ops.paged_attention_decode(q, kv_layer, md.block_tables, md.seq_lens, self.scale,
                                           md.max_seq_len, rope=rope, **self.kv_scales[i])
        elif nd == 0:
            o = ops.paged_attention_prefill(q, kv_layer, md.block_tables, md.query_start_loc,
                                            md.seq_lens, self.scale, md.max_query_len, rope=rope, **self.kv_scales[i])
        else:
            o = torch.empty(q.shape, dtype=q.dtype, device=q.device)
            rd = rp = None
            if rope is not None:
                rd, rp = (md.positions[:nd], self.cos_sin), (md.positions[nd:], self.cos_sin)
            # mixed step: the prefill chunk's attention (MFMA-bound) on a second stream under the
            # decode rows' attention (HBM-bound); both only read the cache written above, and the main
            # stream joins before o_proj (scripts/probes/attn_overlap_probe.py)
            side = self._side_stream(q.device) if _ATTN_OVERLAP else None
            if side is not None:
                main = torch.cuda.current_stream(q.device)
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    ops.paged_attention_prefill(q[nd:], kv_layer, md.block_tables[nd:], md.prefill_query_start_loc,
                                                md.seq_lens[nd:], self.scale, md.max_query_len, out=o[nd:], rope=rp,
                                                **self.kv_scales[i])
            ops.paged_attention_decode(q[:nd], kv_layer, md.block_tables[:nd], md.seq_lens[:nd], self.scale,
                                       md.max_seq_len, out=o[:nd], rope=rd, **self.kv_scales[i])
            if side is not None:
                main.wait_stream(side)
            else:
                ops.paged_attention_prefill(q[nd:], kv_layer, md.block_tables[nd:], md.prefill_query_start_loc,
                                            md.seq_lens[nd:], self.scale, md.max_query_len, out=o[nd:], rope=rp,
                                            **self.kv_scales[i])
        if not project:  # the caller fuses o_proj with the residual add + next norm
            return o.reshape(o.shape[0], -1)
        out = ops.linear(o.reshape(o.shape[0], -1), w[p + "o"])
        return tp_all_reduce(out)

    def _attention_sampled(self, i: int, h: Optional[torch.Tensor], md: AttnMetadata, kv_layer: torch.Tensor,
                           project: bool = True, qkv: Optional[torch.Tensor] = None):
        """Last layer of a step with prefill chunks: K/V of every token still go to the cache, but
        only the rows that produce logits (the last token of each sampled sequence) need attention,
        o_proj and the MLP.  Each such row is a single query at position seq_len - 1 over its whole
        context, i.e. exactly a decode query, so it runs on the decode kernel."""
        c, w, p = self.cfg, self.w, f"l{i}."
        x = h if qkv is None else qkv
        if _SAMPLED_QROPE and self._fused_q_rope(x, i, qkv is not None):
            # K / V of every token into the cache; q stays un-rotated in the qkv rows and only the
            # sampled rows' q is gathered and rotated inside the decode kernel (no [T, Hq, D] q write)
            if qkv is None:
                qkv = ops.linear(h, w[p + "qkv"])
            q = ops.rope_kv_into_cache(qkv, self.nh, self.nkv, self.hd, md.positions, self.cos_sin, kv_layer,
                                       md.slot_mapping, **self.kv_scales[i], num_decodes=md.num_decodes)
            ns = md.logits_indices.shape[0]
            if ns == 0:
                return q.new_empty((0, self.cfg.hidden_size))
            qs = q.index_select(0, md.logits_indices)
            seq = md.sample_seq.long()
            o = ops.paged_attention_decode(qs, kv_layer, md.block_tables.index_select(0, seq),
                                           md.seq_lens.index_select(0, seq), self.scale, md.max_seq_len,
                                           rope=(md.positions.index_select(0, md.logits_indices), self.cos_sin),
                                           **self.kv_scales[i])
            if not project:
                return o.reshape(ns, -1)
            return tp_all_reduce(ops.linear(o.reshape(ns, -1), w[p + "o"]))
        if qkv is not None:
            q = ops.rope_and_cache(qkv, self.nh, self.nkv, self.hd, md.positions, self.cos_sin, kv_layer,
                                   md.slot_mapping, w.get(p + "q_norm"), w.get(p + "k_norm"), c.rms_norm_eps,
                                   **self.kv_scales[i])
        else:
            q = ops.linear_rope_and_cache(h, w[p + "qkv"], self.nh, self.nkv, self.hd, md.positions, self.cos_sin,
                                          kv_layer, md.slot_mapping, w.get(p + "q_norm"), w.get(p + "k_norm"),
                                          c.rms_norm_eps, **self.kv_scales[i])
        ns = md.logits_indices.shape[0]
        if ns == 0:  # no sequence samples this step: the layer only wrote K/V
            return q.new_empty((0, self.cfg.hidden_size))
        qs = q.index_select(0, md.logits_indices)
        seq = md.sample_seq.long()
        bt = md.block_tables.index_select(0, seq)
        sl = md.seq_lens.index_select(0, seq)
        if not q.is_cuda:
            qsl = torch.arange(ns + 1, dtype=torch.int32, device=q.device)
            o = ref.paged_attention(qs, kv_layer, bt, qsl, sl, self.scale, **self.kv_scales[i])
        else:
            o = ops.paged_attention_decode(qs, kv_layer, bt, sl, self.scale, md.max_seq_len, **self.kv_scales[i])
        if not project:
            return o.reshape(ns, -1)
        out = ops.linear(o.reshape(ns, -1), w[p + "o"])
        return tp_all_reduce(out)

    def _mlp(self, i: int, h: torch.Tensor, reduce: bool = True) -> tuple:
        """(output, partial): partial = the output is this rank's share, still to be all-reduced
        (always False when reduce=True: the all-reduce ran here)."""
        w, p = self.w, f"l{i}."
        if self.cfg.is_moe and self.moe_dispatch == "a2a" and self.tp_size > 1:
            from ..parallel.expert import moe_a2a
            return moe_a2a(h, w[p + "gate"], w[p + "w13"], w[p + "w2"], self.cfg.num_experts_per_tok,
                           self.tp_rank, self.tp_size, get_tp().group), False
        if self.cfg.is_moe:
            router = F.linear(h, w[p + "gate"])
            tw, tid = ops.moe_topk_softmax(router, self.cfg.num_experts_per_tok)
            out = ops.moe_experts(h, w[p + "w13"], w[p + "w2"], tw, tid, self.e_offset)
        else:
            a = ops.gate_up_silu(h, w[p + "gate_up"])
            out = ops.linear(a, w[p + "down"])
        if not reduce:
            return out, self.tp_size > 1
        return tp_all_reduce(out), False

    @torch.inference_mode()
    def calibrate_kv_scales(self, block_size: int = 16, n: int = 256, headroom: float = 2.0) -> None:
        """Per-layer K / V scales for an fp8 KV cache from one probe prefill (seeded random tokens,
        bf16 scratch cache): scale = amax / (448 / headroom), so the probe's largest value sits a
        factor `headroom` below the e4m3 limit and small values stay out of the subnormal range
        (vLLM's --calculate-kv-scales idea).  Every worker of a model derives the same scales from
        the same weights, so prefill and decode workers agree on the bytes they exchange."""
        c, dev = self.cfg, self.device
        g = torch.Generator().manual_seed(1234)
        ids = torch.randint(3, c.vocab_size, (n,), generator=g).to(dev)
        nb = -(-n // block_size)
        kv = torch.zeros(nb, c.num_layers, 2, self.nkv, block_size, c.head_dim, dtype=self.dtype, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        pos = torch.arange(n, device=dev)
        qsl = torch.tensor([0, n], **i32)
        md = AttnMetadata(positions=pos, slot_mapping=pos.clone(), block_tables=torch.arange(nb, **i32).unsqueeze(0),
                          seq_lens=torch.tensor([n], **i32), query_start_loc=qsl,
                          logits_indices=torch.tensor([n - 1], device=dev), num_decodes=0, num_prefills=1,
                          num_prefill_tokens=n, max_query_len=n, max_seq_len=n, prefill_query_start_loc=qsl)
        self.forward(ids, md, kv)
        amax = kv.float().abs().amax(dim=(0, 3, 4, 5)).cpu()  # [L, 2]
        lim = 448.0 / headroom
        self.kv_scales = [{"k_scale": max(float(amax[i, 0]) / lim, 1e-8),
                           "v_scale": max(float(amax[i, 1]) / lim, 1e-8)} for i in range(c.num_layers)]

    def embed(self, input_ids: torch.Tensor) -> torch.Tensor:
        return F.embedding(input_ids, self.w["embed"])

    def forward(self, input_ids: torch.Tensor, md: AttnMetadata, kv_cache: torch.Tensor) -> torch.Tensor:
        """Returns final hidden states (normed) of the rows selected by md.logits_indices."""
        c = self.cfg
        # steps with prefill chunks: the last layer only computes the rows that produce logits
        prune = self.prune_last_layer and md.num_prefills > 0 and md.sample_seq is not None
        if self.pf_chain and input_ids.shape[0] > 256 and input_ids.is_cuda and (md.num_prefills > 0 or self.pf_decode):
            return self._forward_pf(input_ids, md, kv_cache, prune)
        # K01: the embedding gather runs inside the first layer's input RMSNorm kernel
        h, residual = ops.embed_rms_norm(input_ids, self.w["embed"], self.w["l0.in_norm"], c.rms_norm_eps)
        if self.fuse_residual and h.is_cuda:
            return self._forward_fused(h, residual, md, kv_cache, prune)
        x = None
        for i in range(c.num_layers):
            p = f"l{i}."
            if i > 0:
                h, residual = ops.fused_add_rms_norm(x, residual, self.w[p + "in_norm"], c.rms_norm_eps)
            if prune and i == c.num_layers - 1:
                x = self._attention_sampled(i, h, md, kv_cache[:, i])
                residual = residual.index_select(0, md.logits_indices)
                if x.shape[0] == 0:  # no sequence samples this step: the layer only wrote K/V
                    return x
            else:
                x = self._attention(i, h, md, kv_cache[:, i])
            h, residual = ops.fused_add_rms_norm(x, residual, self.w[p + "post_norm"], c.rms_norm_eps)
            x = self._mlp(i, h)[0]
        h, _ = ops.fused_add_rms_norm(x, residual, self.w["norm"], c.rms_norm_eps)
        return h if prune else h.index_select(0, md.logits_indices)

    def _forward_fused(self, h: torch.Tensor, residual: torch.Tensor, md: AttnMetadata, kv_cache: torch.Tensor,
                       prune: bool) -> torch.Tensor:
        """Every projection that feeds the residual stream ends in the next RMSNorm, so a layer is
        qkv -> rope/cache -> attention -> o+add+norm -> gate_up+SiLU -> down+add+norm(next layer's
        input norm, or the final norm).  TP = 1: ops.linear_add_rms_norm (split-K slabs summed in the
        norm kernel).  TP > 1: comm.tp_linear_add_rms_norm -- the row-parallel partial (or its split-K
        slabs) goes through ONE kernel that all-reduces over the IPC mesh, adds the residual and
        normalises (custom_allreduce.hip car_add_rmsnorm_kernel)."""
        c, w = self.cfg, self.w
        eps = c.rms_norm_eps
        L = c.num_layers
        for i in range(L):
            p = f"l{i}."
            if prune and i == L - 1:
                o = self._attention_sampled(i, h, md, kv_cache[:, i], project=False)
                if o.shape[0] == 0:  # no sequence samples this step: the layer only wrote K/V
                    return o.new_empty((0, h.shape[1]))
                residual = residual.index_select(0, md.logits_indices)
            else:
                o = self._attention(i, h, md, kv_cache[:, i], project=False)
            h, residual = tp_linear_add_rms_norm(o, w[p + "o"], residual, w[p + "post_norm"], eps)
            nxt = w[f"l{i + 1}.in_norm"] if i + 1 < L else w["norm"]
            if c.is_moe:
                y, partial = self._mlp(i, h, reduce=False)
                h, residual = tp_add_rms_norm(y, residual, nxt, eps) if partial else \
                    ops.fused_add_rms_norm(y, residual, nxt, eps)
            else:
                h, residual = tp_linear_add_rms_norm(ops.gate_up_silu(h, w[p + "gate_up"]), w[p + "down"], residual,
                                                     nxt, eps)
        return h if prune else h.index_select(0, md.logits_indices)

    def _forward_pf(self, input_ids: torch.Tensor, md: AttnMetadata, kv_cache: torch.Tensor,
                    prune: bool) -> torch.Tensor:
        """Prefill / mixed steps (M > 256 rows, TP = 1, dense, GPU).  The residual stream r is the only
        activation between the projections: every RMSNorm runs inside its consumer GEMM (gemm_pf row
        scale over the norm-folded weight, the x^2 row sums taken from the X fragments the tile streams
        anyway) and every residual add inside its producer (gemm_pf epi 2, r updated in place).  A layer
        is qkv(rs) -> rope/cache -> attention -> o(+r) -> gate_up(rs, SwiGLU) -> down(+r): four GEMMs
        and no normalisation pass over [M, hidden].  Per projection and row bucket the start-up tuner
        (ops/prefill_pf.tune_fused) keeps a norm pass + the unfused GEMM, or hipBLASLt addmm_, where
        those measured faster.  The last layer of a pruned step finishes on the sampled rows through
        the unfused decode-size path."""
        from ..ops.prefill_pf import norm_linear, resid_linear
        c, w, wf = self.cfg, self.w, self.wf
        eps = c.rms_norm_eps
        L = c.num_layers
        r = F.embedding(input_ids, w["embed"])
        for i in range(L):
            p = f"l{i}."
            qkv = norm_linear(r, w[p + "qkv"], wf.get(p + "qkv"), w[p + "in_norm"], eps, 0)
            if prune and i == L - 1:
                o = self._attention_sampled(i, None, md, kv_cache[:, i], project=False, qkv=qkv)
                if o.shape[0] == 0:  # no sequence samples this step: the layer only wrote K/V
                    return o.new_empty((0, c.hidden_size))
                rs = r.index_select(0, md.logits_indices)
                h, rs = tp_linear_add_rms_norm(o, w[p + "o"], rs, w[p + "post_norm"], eps)
                return tp_linear_add_rms_norm(ops.gate_up_silu(h, w[p + "gate_up"]), w[p + "down"], rs, w["norm"],
                                              eps)[0]
            o = self._attention(i, None, md, kv_cache[:, i], project=False, qkv=qkv)
            resid_linear(o, w[p + "o"], r)
            m = norm_linear(r, w[p + "gate_up"], wf.get(p + "gate_up"), w[p + "post_norm"], eps, 1)
            resid_linear(m, w[p + "down"], r)
        return ops.rms_norm(r.index_select(0, md.logits_indices), w["norm"], eps)

    def compute_logits(self, hidden: torch.Tensor) -> torch.Tensor:
        # bf16 on the GPU: the sampling kernel reads bf16 rows directly (no fp32 copy of [B, V])
        logits = ops.linear(hidden, self.lm_head_weight())
        if self.tp_size > 1:
            logits = tp_all_gather(logits, dim=-1)
        return logits[:, :self.cfg.vocab_size]


_FUSED_Q_ROPE = os.environ.get("MXS_FUSED_Q_ROPE", "1") == "1"
_SAMPLED_QROPE = os.environ.get("MXS_SAMPLED_QROPE", "1") == "1"  # pruned last layer: q rotated in-kernel
_ATTN_OVERLAP = os.environ.get("MXS_ATTN_OVERLAP", "1") == "1"  # mixed steps: prefill attention on a side stream


def _pad_rows(t: torch.Tensor, n: int) -> torch.Tensor:
    if t.shape[0] >= n:
        return t
    pad = torch.zeros((n - t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    return torch.cat([t, pad])


def build_model(cfg: ModelConfig, device, dtype=torch.bfloat16, moe_dispatch: str = "allreduce") -> TransformerLM:
    return TransformerLM(cfg, device, dtype, moe_dispatch)
