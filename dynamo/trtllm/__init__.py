"""`python3 -m dynamo.trtllm`: mxserve worker accepting the trtllm flag dialect."""
