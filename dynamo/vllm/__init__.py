"""`python3 -m dynamo.vllm`: mxserve worker accepting the vllm flag dialect."""
