"""Contiguous sharding of a descriptor batch over GPUs / ranks.

Same split as the C shim (fd_ed25519_gpu_submit: shard i of N covers
[n*i/N, n*(i+1)/N)).  Signatures are independent, so no txn alignment and no
collective is needed: results are concatenated in shard order (the host-side
gather of SURVEY.md §8(e))."""


def shard_range(n, i, parts):
    return n * i // parts, n * (i + 1) // parts
