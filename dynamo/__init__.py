"""Drop-in module names for the reference manifests: `python3 -m dynamo.vllm|sglang|trtllm|frontend`
(examples/deploy/*/agg.yaml:29-32) start this framework's worker / frontend with the matching flag
dialect.  Nothing here imports NVIDIA Dynamo."""
