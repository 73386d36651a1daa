"""Benchmark harness shipped in-repo (replaces `benchmarks.utils.benchmark` from upstream Dynamo +
aiperf, which the reference clones at setup time: run-benchmarks.sh:61-71)."""
