"""`python3 -m dynamo.frontend`: the mxserve OpenAI frontend."""
