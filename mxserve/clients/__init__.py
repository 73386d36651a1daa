"""Client tools behind the drop-in scripts (chat.sh, multi_convos_parallel.sh)."""
