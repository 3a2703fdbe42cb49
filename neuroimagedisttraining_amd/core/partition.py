"""Non-IID client partitioners.

Semantics follow the reference; implementations are new:

* ``dir``      — per-client Dirichlet class prior, equal quotas, sequential draws taking the last
                 remaining index of the drawn class (``cifar10/data_loader.py:118-149``).
* ``n_cls``    — each client gets a uniform prior over ``int(alpha)`` random classes; an exhausted
                 class is *refilled* to a random level, so samples can repeat (``:80-116``).
* ``my_part``  — clients share ``Dir(0.3)`` priors in shards; exhausted classes reset to full
                 (``:151-191``).
* ``homo``     — random permutation split evenly (``tiny_imagenet/data_loader.py:87-91``).
* ``hetero``   — FedML LDA with balance cap and ``min_size`` retries
                 (``fedml_core/non_iid_partition/noniid_partition.py:6-73``).
* ``site``     — one client per acquisition site with a seeded 80/20 split
                 (``ABCD/data_loader.py:74-87``).

All functions take an explicit ``numpy.random.RandomState`` (default: the global one, which is
what the reference seeds) so runs are reproducible.
"""
from __future__ import annotations

import logging
import math

import numpy as np

__all__ = [
    "partition_dir", "partition_n_cls", "partition_my_part", "partition_homo", "partition_hetero",
    "non_iid_partition_with_dirichlet_distribution",
    "partition_class_samples_with_dirichlet_distribution", "record_data_stats", "partition_by_site",
    "partition_labels", "per_client_test_indices", "equal_quotas",
]


def _rs(rng):
    return np.random.mtrand._rand if rng is None else rng


def equal_quotas(n_samples: int, n_clients: int) -> np.ndarray:
    """lognormal(log(N/C), sigma=0) normalised then truncated == equal integer quotas."""
    per = np.full(n_clients, n_samples / n_clients)
    return (per / per.sum() * n_samples).astype(np.int64)


def _sequential_prior_draw(labels, n_clients, priors, n_cls, rng, exhausted):
    """Shared sampler for dir / n_cls / my_part.

    ``exhausted`` selects what happens when the drawn class has no indices left:
    ``"redraw"`` (dir), ``"random_refill"`` (n_cls) or ``"full_refill"`` (my_part).
    """
    rng = _rs(rng)
    quota = equal_quotas(len(labels), n_clients)
    cdf = np.cumsum(priors, axis=1)
    by_cls = [np.where(labels == c)[0] for c in range(n_cls)]
    left = np.array([len(ix) for ix in by_cls], dtype=np.int64)
    out = [[] for _ in range(n_clients)]
    remaining = int(quota.sum())
    while remaining > 0:
        c = int(rng.randint(n_clients))
        if quota[c] <= 0:
            continue
        quota[c] -= 1
        remaining -= 1
        row = cdf[c]
        tries = 0
        while True:
            tries += 1
            if tries > 1000 and exhausted == "redraw":
                # The reference redraws forever when a client's prior has (numerically) no mass left on any
                # class with remaining samples; after 1000 misses draw from the prior restricted to
                # non-exhausted classes instead (identical behaviour whenever the reference terminates quickly).
                pr = priors[c] * (left > 0)
                pr = pr / pr.sum() if pr.sum() > 0 else (left > 0) / max(1, int((left > 0).sum()))
                row = np.cumsum(pr)
                tries = -10 ** 9
            k = int(np.argmax(rng.uniform() <= row))
            if left[k] <= 0:
                if exhausted == "random_refill":
                    left[k] = rng.randint(0, len(by_cls[k]))
                elif exhausted == "full_refill":
                    left[k] = len(by_cls[k])
                if len(by_cls[k]) == 0 and exhausted != "redraw":
                    raise ValueError("class %d has no samples" % k)
                continue
            left[k] -= 1
            out[c].append(int(by_cls[k][left[k]]))
            break
    return {i: np.asarray(v, dtype=np.int64) for i, v in enumerate(out)}


def partition_dir(labels, n_clients, alpha, n_cls=None, rng=None):
    labels = np.asarray(labels)
    n_cls = int(labels.max()) + 1 if n_cls is None else n_cls
    priors = _rs(rng).dirichlet([alpha] * n_cls, size=n_clients)
    return _sequential_prior_draw(labels, n_clients, priors, n_cls, rng, "redraw")


def partition_n_cls(labels, n_clients, alpha, n_cls=None, rng=None):
    labels = np.asarray(labels)
    n_cls = int(labels.max()) + 1 if n_cls is None else n_cls
    r = _rs(rng)
    k = int(alpha)
    priors = np.zeros((n_clients, n_cls))
    for i in range(n_clients):
        priors[i, r.choice(n_cls, k, replace=False)] = 1.0 / alpha
    return _sequential_prior_draw(labels, n_clients, priors, n_cls, rng, "random_refill")


def partition_my_part(labels, n_clients, alpha, n_cls=None, rng=None):
    """Shard-shared Dir(0.3) priors.  ``alpha`` is the number of shards per client fraction; the
    CIFAR-10 variant (``int(alpha*C)`` priors indexed ``i // int(C/alpha)``) is used."""
    labels = np.asarray(labels)
    n_cls = int(labels.max()) + 1 if n_cls is None else n_cls
    r = _rs(rng)
    n_prior = max(1, int(alpha * n_clients))
    tmp = r.dirichlet([0.3] * n_cls, size=n_prior)
    stride = max(1, int(n_clients / alpha))
    priors = np.stack([tmp[min(i // stride, n_prior - 1)] for i in range(n_clients)])
    return _sequential_prior_draw(labels, n_clients, priors, n_cls, rng, "full_refill")


def partition_homo(n_samples, n_clients, rng=None):
    perm = _rs(rng).permutation(n_samples)
    return {i: np.asarray(p, dtype=np.int64) for i, p in enumerate(np.array_split(perm, n_clients))}


def partition_class_samples_with_dirichlet_distribution(N, alpha, client_num, idx_batch, idx_k, rng=None):
    r = _rs(rng)
    r.shuffle(idx_k)
    props = r.dirichlet(np.repeat(alpha, client_num))
    cap = np.array([len(b) < N / client_num for b in idx_batch], dtype=np.float64)
    props = props * cap
    props = props / props.sum()
    cuts = (np.cumsum(props) * len(idx_k)).astype(int)[:-1]
    idx_batch = [b + part.tolist() for b, part in zip(idx_batch, np.split(idx_k, cuts))]
    return idx_batch, min(len(b) for b in idx_batch)


def non_iid_partition_with_dirichlet_distribution(label_list, client_num, classes, alpha,
                                                  task="classification", min_size_required=10, rng=None):
    """FedML LDA partitioner (``noniid_partition.py:6-73``)."""
    r = _rs(rng)
    N = len(label_list) if task == "segmentation" else np.asarray(label_list).shape[0]
    min_size = 0
    while min_size < min_size_required:
        idx_batch = [[] for _ in range(client_num)]
        if task == "segmentation":
            for c, cat in enumerate(classes):
                seen = set(classes[:c])
                idx_k = np.asarray([i for i in range(len(label_list))
                                    if np.any(np.asarray(label_list[i]) == cat)
                                    and not any(x in seen for x in np.ravel(label_list[i]))], dtype=np.int64)
                idx_batch, min_size = partition_class_samples_with_dirichlet_distribution(
                    N, alpha, client_num, idx_batch, idx_k, r)
        else:
            labels = np.asarray(label_list)
            for k in range(classes):
                idx_k = np.where(labels == k)[0]
                idx_batch, min_size = partition_class_samples_with_dirichlet_distribution(
                    N, alpha, client_num, idx_batch, idx_k, r)
    out = {}
    for i in range(client_num):
        b = np.asarray(idx_batch[i], dtype=np.int64)
        r.shuffle(b)
        out[i] = b
    return out


def partition_hetero(labels, n_clients, alpha, n_cls=None, min_size_required=10, rng=None):
    labels = np.asarray(labels)
    n_cls = int(labels.max()) + 1 if n_cls is None else n_cls
    return non_iid_partition_with_dirichlet_distribution(labels, n_clients, n_cls, alpha,
                                                         min_size_required=min_size_required, rng=rng)


def record_data_stats(y_train, net_dataidx_map, task="classification"):
    y_train = np.asarray(y_train, dtype=object) if task == "segmentation" else np.asarray(y_train)
    stats = {}
    for i, idx in net_dataidx_map.items():
        vals = np.concatenate([np.ravel(y_train[j]) for j in idx]) if task == "segmentation" else y_train[idx]
        u, c = np.unique(vals, return_counts=True)
        stats[i] = {int(a): int(b) for a, b in zip(u, c)}
    logging.debug("Data statistics: %s", stats)
    return stats


def partition_by_site(site, split_ratio=0.2, seed=42, max_clients=None):
    """ABCD site-as-client split: for every unique site, shuffle its indices with ``seed`` and
    keep the first ``len - int(len*split_ratio)`` for training (``ABCD/data_loader.py:74-87``).

    Returns ``(train_map, test_map, site_values)``; ``max_clients`` reproduces the reference's
    hard-coded first-21-sites behaviour (quirk Q9) when set to 21.
    """
    site = np.asarray(site)
    train, test, values = {}, {}, []
    for ci, s in enumerate(np.unique(site)):
        if max_clients is not None and ci >= max_clients:
            break
        ix = np.where(site == s)[0]
        n_test = int(len(ix) * split_ratio)
        r = np.random.RandomState(seed)
        ix = ix.copy()
        r.shuffle(ix)
        n_train = len(ix) - n_test
        train[ci], test[ci] = ix[:n_train], ix[n_train:]
        values.append(s)
    return train, test, values


def partition_labels(method, labels, n_clients, alpha, n_cls=None, rng=None):
    """Dispatch by the reference's ``--partition_method`` names."""
    if method == "dir":
        return partition_dir(labels, n_clients, alpha, n_cls, rng)
    if method == "n_cls":
        return partition_n_cls(labels, n_clients, alpha, n_cls, rng)
    if method == "my_part":
        return partition_my_part(labels, n_clients, alpha, n_cls, rng)
    if method == "homo":
        return partition_homo(len(labels), n_clients, rng)
    if method == "hetero":
        return partition_hetero(labels, n_clients, alpha, n_cls, rng=rng)
    raise ValueError("unknown partition method %r" % method)


def per_client_test_indices(train_labels, test_labels, train_map, n_cls=None, rng=None):
    """Per-client test sets drawn proportionally to each client's train label histogram:
    for class c, ``ceil(count_c / total * ceil(|test| / C))`` random test indices of class c, C = the number of
    clients (``tmp_tst_num`` of ``cifar10/data_loader.py:226-236``, the same in the cifar100 / tiny_imagenet / ABCD
    loaders): about |test| / C samples per client (100 for CIFAR-10 with 100 clients).  Test sets may overlap across
    clients.  (Rounds 1-5 divided by the class count instead: CIFAR-10 clients got ~1000 test samples each, ten
    times the reference's evaluation work.)"""
    r = _rs(rng)
    train_labels, test_labels = np.asarray(train_labels), np.asarray(test_labels)
    n_cls = int(max(train_labels.max(), test_labels.max())) + 1 if n_cls is None else n_cls
    by_cls = [np.where(test_labels == c)[0] for c in range(n_cls)]
    per_client = math.ceil(len(test_labels) / max(1, len(train_map)))
    out = {}
    for i, idx in train_map.items():
        hist = np.bincount(train_labels[idx], minlength=n_cls)
        tot = max(1, hist.sum())
        pick = []
        for c in range(n_cls):
            n = math.ceil(hist[c] / tot * per_client)
            if n > 0 and len(by_cls[c]) > 0:
                pick.append(r.choice(by_cls[c], min(n, len(by_cls[c])), replace=False))
        out[i] = np.concatenate(pick).astype(np.int64) if pick else np.zeros(0, np.int64)
    return out
