"""FedML-compatible core API (compat surface over neuroimagedisttraining_amd)."""
