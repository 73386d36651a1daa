"""Request state and sampling parameters."""
from __future__ import annotations

import enum
import time
from dataclasses import dataclass, field
from typing import Optional


@dataclass
class SamplingParams:
    max_tokens: int = 16
    temperature: float = 1.0
    top_p: float = 1.0
    top_k: int = 0
    seed: Optional[int] = None
    stop_token_ids: list = field(default_factory=list)
    ignore_eos: bool = False
    min_tokens: int = 0
    # log-probs of the sampled tokens: None = off, k >= 0 = also the k most likely tokens (k <= 20)
    logprobs: Optional[int] = None
    repetition_penalty: float = 1.0  # > 1 discourages tokens of the prompt and the output (vLLM)
    frequency_penalty: float = 0.0  # OpenAI: minus count * value for generated tokens
    presence_penalty: float = 0.0  # OpenAI: minus value once a token was generated

    @property
    def has_penalties(self) -> bool:
        return self.repetition_penalty != 1.0 or self.frequency_penalty != 0.0 or self.presence_penalty != 0.0

    @classmethod
    def from_openai(cls, body: dict, default_max_tokens: int = 256) -> "SamplingParams":
        mt = body.get("max_completion_tokens", body.get("max_tokens"))
        temp = body.get("temperature")
        return cls(
            max_tokens=int(mt) if mt is not None else default_max_tokens,
            temperature=1.0 if temp is None else float(temp),
            top_p=float(body.get("top_p", 1.0) if body.get("top_p") is not None else 1.0),
            top_k=int(body.get("top_k", 0) or 0),
            seed=body.get("seed"),
            stop_token_ids=list(body.get("stop_token_ids") or []),
            ignore_eos=bool(body.get("ignore_eos", False)),
            min_tokens=int(body.get("min_tokens", 0) or 0),
            logprobs=body.get("logprobs"),
            repetition_penalty=float(body.get("repetition_penalty") or 1.0),
            frequency_penalty=float(body.get("frequency_penalty") or 0.0),
            presence_penalty=float(body.get("presence_penalty") or 0.0),
        )


class Status(enum.Enum):
    WAITING = "waiting"
    RUNNING = "running"
    PREEMPTED = "preempted"
    FINISHED_STOPPED = "stop"
    FINISHED_LENGTH = "length"
    FINISHED_ABORTED = "abort"

    @property
    def finished(self) -> bool:
        return self in (Status.FINISHED_STOPPED, Status.FINISHED_LENGTH, Status.FINISHED_ABORTED)


_seed_counter = 0


def _next_seed() -> int:
    global _seed_counter
    _seed_counter += 1
    return (int(time.time_ns()) ^ (_seed_counter * 0x9E3779B1)) & 0x7FFFFFFF


@dataclass
class Request:
    request_id: str
    prompt_token_ids: list
    sampling: SamplingParams = field(default_factory=SamplingParams)
    arrival_time: float = field(default_factory=time.monotonic)
    eos_token_ids: tuple = ()
    # disaggregation: "prefill_only" stops after the first token and keeps the KV blocks pinned
    # for transfer; "remote_prefill" expects KV for the prompt to be written by a prefill worker.
    disagg_role: Optional[str] = None

    output_token_ids: list = field(default_factory=list)
    status: Status = Status.WAITING
    num_computed_tokens: int = 0
    num_cached_tokens: int = 0
    block_ids: list = field(default_factory=list)
    block_hashes: list = field(default_factory=list)
    num_registered_blocks: int = 0
    seed: int = 0
    submit_time: Optional[float] = None  # monotonic: the serving layer received it (before the engine inbox)
    scheduled_time: Optional[float] = None  # first admitted into a step (queue time ends)
    first_token_time: Optional[float] = None
    finish_time: Optional[float] = None
    num_preemptions: int = 0
    kv_gen: int = 0  # bumped whenever block_ids is rebuilt from scratch (free / preempt)
    # tokens scheduled for sampling whose value is still on the GPU (async scheduling: step N+1 is
    # scheduled before step N's sampled ids reach the host; a decode's input is then read on the
    # device from the row's last sampled token)
    num_pending: int = 0
    # prefill_only on the GPU: an event recorded right after the launch of the step that wrote the
    # prompt's last KV block -- a KV push waits on it, not on everything queued behind that step
    kv_ready: Optional[object] = None

    def __post_init__(self):
        self.seed = self.sampling.seed if self.sampling.seed is not None else _next_seed()

    @property
    def num_prompt_tokens(self) -> int:
        return len(self.prompt_token_ids)

    @property
    def num_tokens(self) -> int:
        """Tokens the sequence will hold once in-flight samples land (scheduling view)."""
        return len(self.prompt_token_ids) + len(self.output_token_ids) + self.num_pending

    @property
    def num_known_tokens(self) -> int:
        return len(self.prompt_token_ids) + len(self.output_token_ids)

    def can_grow(self, max_model_len: int) -> bool:
        """False once the in-flight samples already reach max_tokens / the context limit."""
        n_out = len(self.output_token_ids) + self.num_pending
        return n_out < self.sampling.max_tokens and self.num_tokens < max_model_len

    def token_at(self, i: int) -> int:
        n = len(self.prompt_token_ids)
        return self.prompt_token_ids[i] if i < n else self.output_token_ids[i - n]

    def all_token_ids(self) -> list:
        return self.prompt_token_ids + self.output_token_ids

    @property
    def is_finished(self) -> bool:
        return self.status.finished

    def check_stop(self, max_model_len: int) -> Optional[Status]:
        n_out = len(self.output_token_ids)
        if n_out == 0:
            return None
        last = self.output_token_ids[-1]
        if n_out >= self.sampling.min_tokens:
            if not self.sampling.ignore_eos and last in self.eos_token_ids:
                return Status.FINISHED_STOPPED
            if last in self.sampling.stop_token_ids:
                return Status.FINISHED_STOPPED
        if n_out >= self.sampling.max_tokens or self.num_known_tokens >= max_model_len:
            return Status.FINISHED_LENGTH
        return None
