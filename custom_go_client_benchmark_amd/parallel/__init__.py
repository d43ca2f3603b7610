"""One reader process per GPU: rendezvous, RCCL barriers, stat reductions."""
