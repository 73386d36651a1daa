"""`python3 -m dynamo.sglang`: mxserve worker accepting the sglang flag dialect."""
