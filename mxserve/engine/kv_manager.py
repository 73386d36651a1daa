"""Per-request KV block bookkeeping on top of the native BlockPool (csrc/runtime/block_pool.cpp).

Prefix caching: every full 16-token block of a request gets a chained hash (same function the
frontend router uses, so KV events line up); a new request reuses the longest run of cached blocks.
"""
from __future__ import annotations

from .. import _native
from .request import Request


class KVCacheManager:
    def __init__(self, num_blocks: int, block_size: int = 16, enable_prefix_caching: bool = True):
        rt = _native.rt()
        self.block_size = block_size
        self.pool = rt.BlockPool(num_blocks, enable_prefix_caching)
        self.caching = enable_prefix_caching
        self._hash = rt.block_hashes

    @property
    def num_blocks(self) -> int:
        return self.pool.num_blocks

    def num_free(self) -> int:
        return self.pool.num_free()

    def usage(self) -> float:
        return self.pool.usage()

    def _update_hashes(self, req: Request) -> None:
        """Extend req.block_hashes to cover every full block of known tokens."""
        bs = self.block_size
        have = len(req.block_hashes)
        want = req.num_known_tokens // bs
        if want <= have:
            return
        parent = req.block_hashes[-1] if have else 0
        toks = req.all_token_ids()[have * bs: want * bs]
        req.block_hashes.extend(self._hash(toks, bs, 0, parent))

    def get_computed_blocks(self, req: Request) -> int:
        """Attach the longest cached prefix to a fresh request; returns the cached token count.
        At least one prompt token is always recomputed (it produces the first logits)."""
        if not self.caching or req.block_ids:
            return 0
        self._update_hashes(req)
        max_blocks = (req.num_tokens - 1) // self.block_size
        hashes = req.block_hashes[:max_blocks]
        if not hashes:
            return 0
        blocks = self.pool.get_cached_prefix(hashes)
        req.block_ids = list(blocks)
        req.num_registered_blocks = len(blocks)
        return len(blocks) * self.block_size

    def allocate_slots(self, req: Request, num_new_tokens: int) -> bool:
        """Ensure blocks for num_computed + num_new tokens.  False if the pool is exhausted."""
        need_tokens = req.num_computed_tokens + num_new_tokens
        if need_tokens <= len(req.block_ids) * self.block_size:  # common decode case
            return True
        need_blocks = -(-need_tokens // self.block_size) - len(req.block_ids)
        if need_blocks <= 0:
            return True
        if need_blocks > self.pool.num_free():
            return False
        req.block_ids.extend(self.pool.allocate(need_blocks))
        return True

    def cache_computed_blocks(self, req: Request, upto: int | None = None) -> None:
        """Register hashes of blocks whose tokens are all computed (becomes reusable by others).
        `upto` caps the computed-token count: with async scheduling num_computed_tokens already
        counts the step still in flight, whose KV is not written yet."""
        if not self.caching:
            return
        done = req.num_computed_tokens if upto is None else min(upto, req.num_computed_tokens)
        full = done // self.block_size
        if full <= req.num_registered_blocks:
            return
        self._update_hashes(req)
        full = min(full, len(req.block_hashes), len(req.block_ids))
        lo = req.num_registered_blocks
        if full > lo:
            self.pool.cache_blocks(req.block_ids[lo:full], req.block_hashes[lo:full])
            req.num_registered_blocks = full

    def free(self, req: Request) -> None:
        if req.block_ids:
            self.pool.free(list(reversed(req.block_ids)))
        req.block_ids = []
        req.num_registered_blocks = 0
        req.kv_gen += 1

    def take_events(self):
        return self.pool.take_events()

    def hit_rate(self) -> float:
        return self.pool.hit_rate()

    def check_invariants(self) -> bool:
        return self.pool.check_invariants()

    def count_prefix_hits(self, token_ids: list) -> int:
        hashes = self._hash(token_ids, self.block_size, 0, 0)
        return self.pool.count_cached_prefix(hashes)


def blocks_needed(num_tokens: int, block_size: int) -> int:
    return -(-num_tokens // block_size)

