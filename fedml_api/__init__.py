"""FedML-compatible API package (compat surface over neuroimagedisttraining_amd)."""
