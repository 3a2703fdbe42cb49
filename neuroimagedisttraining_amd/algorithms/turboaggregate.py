"""Secure-aggregation building blocks (reference ``fedml_api/standalone/turboaggregate/{mpc_function,TA_trainer,
TA_client}.py``) and a working secure FedAvg.

Finite-field helpers over a prime ``p`` (int64 numpy; p < 2**31 so products fit): modular inverse, Lagrange
coefficients, BGW (Shamir) encoding/decoding, Lagrange Coded Computing (LCC) encoding/decoding, additive secret
sharing and a toy Diffie-Hellman key agreement.  The reference's trainer hook is a ``pass`` stub; here
:class:`TurboAggregateTrainer` runs an actual secure aggregation round: every client quantises its weighted
update to fixed point in Z_p, adds pairwise masks derived from agreed keys (they cancel in the sum), the server
sums the masked vectors and de-quantises — the result equals plain FedAvg up to the quantisation step, and the
server never sees an individual client's vector.  Dropped clients' masks are recovered from BGW shares of their
secret keys held by the survivors.
"""
from __future__ import annotations

import numpy as np

P_DEFAULT = 2 ** 31 - 1  # Mersenne prime


def modular_inv(a, p):
    """a^-1 mod p (p prime) by Fermat."""
    return pow(int(a) % p, p - 2, p)


def divmod(_num, _den, _p):  # noqa: A001 (reference name)
    return (int(_num) % _p) * modular_inv(_den, _p) % _p


def PI(vals, p):  # noqa: N802
    acc = 1
    for v in vals:
        acc = acc * (int(v) % p) % p
    return acc


def gen_Lagrange_coeffs(alpha_s, beta_s, p, is_K1=0):  # noqa: N802
    """U[i][j] = prod_{o != beta_j} (alpha_i - o) / (beta_j - o)  (mod p)."""
    alphas = [alpha_s[0]] if is_K1 == 1 else list(alpha_s)
    U = np.zeros((len(alphas), len(beta_s)), dtype=np.int64)
    for i, a in enumerate(alphas):
        for j, b in enumerate(beta_s):
            others = [o for o in beta_s if o != b]
            U[i, j] = divmod(PI([a - o for o in others], p), PI([b - o for o in others], p), p)
    return U


# model-sized encodings (U [N x K] @ X [K x d], d in the millions) go to the gfx950 kernel when a GPU is present
DEVICE_MIN_ELEMS = 1 << 16


def matmul_mod_device(A, B, p, device="cuda"):
    """(A @ B) mod p on the GPU (``mpc.hip`` ``modp_matmul``): int64 operands reduced to [0, p), p < 2^32."""
    import torch
    from .. import ops
    A = torch.as_tensor(np.asarray(A, dtype=np.int64) % p).to(device).contiguous()
    B = torch.as_tensor(np.asarray(B, dtype=np.int64) % p).to(device).contiguous()
    C = torch.empty((A.shape[0], B.shape[1]), dtype=torch.int64, device=device)
    ops.ext().modp_matmul(A.data_ptr(), B.data_ptr(), C.data_ptr(), A.shape[0], A.shape[1], B.shape[1], int(p),
                          ops.stream())
    return C.cpu().numpy()


def _matmul_mod(A, B, p):
    """(A @ B) mod p without int64 overflow (row-by-row accumulation of reduced products); large products on the
    GPU kernel."""
    A = np.asarray(A, dtype=np.int64) % p
    B = np.asarray(B, dtype=np.int64) % p
    if B.size >= DEVICE_MIN_ELEMS and p < (1 << 32):
        import torch
        if torch.cuda.is_available():
            return matmul_mod_device(A, B, p)
    out = np.zeros((A.shape[0], B.shape[1]), dtype=np.int64)
    for k in range(A.shape[1]):
        out = (out + (A[:, k:k + 1] * B[k:k + 1, :]) % p) % p
    return out


def BGW_encoding(X, N, T, p, rng=None):  # noqa: N802
    """Shamir shares of X (shape [m, d]) for N workers, threshold T: f(a) = X + sum_t R_t a^t at a = 1..N."""
    rng = np.random if rng is None else rng
    X = np.asarray(X, dtype=np.int64) % p
    R = rng.randint(p, size=(T,) + X.shape).astype(np.int64)
    out = np.zeros((N,) + X.shape, dtype=np.int64)
    for n in range(N):
        a = n + 1
        acc = X.copy()
        ap = 1
        for t in range(T):
            ap = ap * a % p
            acc = (acc + R[t] * ap) % p
        out[n] = acc
    return out


def gen_BGW_lambda_s(alpha_s, p):  # noqa: N802
    """Lagrange coefficients that interpolate f(0) from evaluations at alpha_s."""
    return gen_Lagrange_coeffs([0], list(alpha_s), p)[0]


def BGW_decoding(f_eval, worker_idx, p):  # noqa: N802
    """Recover f(0) from >= T+1 shares; ``worker_idx`` are 0-based worker ids (evaluation points idx+1)."""
    lam = gen_BGW_lambda_s([int(i) + 1 for i in worker_idx], p)
    f = np.asarray(f_eval, dtype=np.int64) % p
    acc = np.zeros(f.shape[1:], dtype=np.int64)
    for k, l in enumerate(lam):
        acc = (acc + f[k] * int(l)) % p
    return acc


def LCC_encoding_with_points(X, alpha_s, beta_s, p):  # noqa: N802
    """Encode the rows X[j] (placed at beta_j) and evaluate the interpolant at alpha_s."""
    U = gen_Lagrange_coeffs(alpha_s, beta_s, p)
    X = np.asarray(X, dtype=np.int64)
    flat = X.reshape(X.shape[0], -1)
    return _matmul_mod(U, flat, p).reshape((len(alpha_s),) + X.shape[1:])


def LCC_decoding_with_points(f_eval, eval_points, target_points, p):  # noqa: N802
    return LCC_encoding_with_points(f_eval, target_points, eval_points, p)


def lcc_points(n, p):
    """The reference's evaluation points: n consecutive integers centred on 0, mod p
    (``stt = -floor(n/2)``, ``mpc_function.py:121-125``)."""
    s = -int(np.floor(n / 2))
    return [int(v) % p for v in range(s, s + n)]


def LCC_encoding(X, N, K, T, p, rng=None):  # noqa: N802
    """Split X [m, d] into K row blocks, append T random blocks, LCC-encode for N workers.  Data blocks sit at the
    reference's centred points beta (K + T of them) and worker j evaluates at the centred point alpha_j (N of
    them), so the shares equal the reference's (``mpc_function.py:111-135``)."""
    rng = np.random if rng is None else rng
    X = np.asarray(X, dtype=np.int64) % p
    m = X.shape[0] // K
    blocks = [X[i * m:(i + 1) * m] for i in range(K)] + [rng.randint(p, size=(m,) + X.shape[1:]) for _ in range(T)]
    return LCC_encoding_with_points(np.stack(blocks), lcc_points(N, p), lcc_points(K + T, p), p)


def LCC_encoding_w_Random(X, R_, N, K, T, p):  # noqa: N802
    X = np.asarray(X, dtype=np.int64) % p
    m = X.shape[0] // K
    blocks = [X[i * m:(i + 1) * m] for i in range(K)] + [np.asarray(R_[t], dtype=np.int64) for t in range(T)]
    return LCC_encoding_with_points(np.stack(blocks), lcc_points(N, p), lcc_points(K + T, p), p)


def LCC_encoding_w_Random_partial(X, R_, N, K, T, p, worker_idx):  # noqa: N802
    return LCC_encoding_w_Random(X, R_, N, K, T, p)[list(worker_idx)]


def LCC_decoding(f_eval, f_deg, N, K, T, worker_idx, p):  # noqa: N802
    """Interpolate the K data blocks from the evaluations of workers ``worker_idx`` (reference
    ``mpc_function.py:195-212``: targets are the K centred points, sources the workers' centred points).  As in
    the reference, the targets coincide with the encoder's first K points only when floor(K/2) ==
    floor((K+T)/2) (e.g. T = 1 with even K); :func:`LCC_decoding_with_points` takes explicit points."""
    if (K // 2) != ((K + T) // 2):
        import warnings
        warnings.warn("LCC_decoding(K=%d, T=%d): the reference's targets lcc_points(K) differ from the encoder's data "
                      "points; use LCC_decode_blocks to recover the encoded blocks" % (K, T), stacklevel=2)
    alpha = lcc_points(N, p)
    ev = [alpha[int(i)] for i in worker_idx]
    need = (K + T - 1) * f_deg + 1
    return LCC_decoding_with_points(np.asarray(f_eval)[:need], ev[:need], lcc_points(K, p), p)


def LCC_decode_blocks(f_eval, f_deg, N, K, T, worker_idx, p):  # noqa: N802
    """Recover the K data blocks that :func:`LCC_encoding` placed at its first K points beta (of K + T) from the
    evaluations of workers ``worker_idx`` — the decoder that matches the encoder for every K, T (the
    reference-compatible :func:`LCC_decoding` does only when floor(K/2) == floor((K+T)/2))."""
    alpha = lcc_points(N, p)
    ev = [alpha[int(i)] for i in worker_idx]
    need = (K + T - 1) * f_deg + 1
    return LCC_decoding_with_points(np.asarray(f_eval)[:need], ev[:need], lcc_points(K + T, p)[:K], p)


def Gen_Additive_SS(d, n_out, p, rng=None):  # noqa: N802
    """n_out additive shares of zero-sum over Z_p (rows sum to 0 mod p)."""
    rng = np.random if rng is None else rng
    s = rng.randint(p, size=(n_out - 1, d)).astype(np.int64)
    last = (-s.sum(0)) % p
    return np.concatenate([s, last[None]], 0)


def my_pk_gen(my_sk, p, g):
    return my_sk if g == 0 else pow(int(g), int(my_sk), p)


def my_key_agreement(my_sk, u_pk, p, g):
    return int(my_sk) * int(u_pk) % p if g == 0 else pow(int(u_pk), int(my_sk), p)


# ------------------------------------------------------------------------------------------------ secure FedAvg
def quantize(v, scale, p):
    q = np.round(np.asarray(v, dtype=np.float64) * scale).astype(np.int64)
    return q % p


def dequantize(q, scale, p):
    q = np.asarray(q, dtype=np.int64) % p
    q = np.where(q > p // 2, q - p, q)
    return q.astype(np.float64) / scale


class TurboAggregateTrainer:
    """Secure FedAvg over flat parameter vectors with pairwise masking and BGW-protected secret keys."""

    def __init__(self, n_clients, p=P_DEFAULT, g=7, scale=2 ** 16, threshold=None, seed=0):
        self.n, self.p, self.g, self.scale = n_clients, p, g, scale
        self.T = threshold if threshold is not None else max(1, n_clients // 2)
        self.rng = np.random.RandomState(seed)
        self.sk = self.rng.randint(1, p - 1, size=n_clients)
        self.pk = [my_pk_gen(s, p, g) for s in self.sk]
        # each client's secret key is Shamir-shared with everyone (for dropout recovery)
        self.sk_shares = [BGW_encoding(np.array([[s]]), n_clients, self.T, p, self.rng) for s in self.sk]

    def _mask(self, i, j, d):
        key = my_key_agreement(self.sk[i], self.pk[j], self.p, self.g)
        r = np.random.RandomState(key % (2 ** 32)).randint(self.p, size=d).astype(np.int64)
        return r if i < j else (-r) % self.p

    def client_upload(self, i, vec, weight):
        d = vec.size
        y = quantize(vec * weight, self.scale, self.p)
        for j in range(self.n):
            if j != i:
                y = (y + self._mask(i, j, d)) % self.p
        return y

    def server_aggregate(self, uploads, dropped=()):
        """``uploads``: dict client -> masked vector.  Masks of dropped clients are removed by reconstructing
        their secret keys from BGW shares held by the survivors."""
        alive = sorted(uploads)
        d = next(iter(uploads.values())).size
        s = np.zeros(d, dtype=np.int64)
        for i in alive:
            s = (s + uploads[i]) % self.p
        for k in dropped:
            shares = np.stack([self.sk_shares[k][i] for i in alive[:self.T + 1]])
            sk_k = int(BGW_decoding(shares, alive[:self.T + 1], self.p)[0, 0])
            assert sk_k == int(self.sk[k])
            for i in alive:  # the survivors' masks with k did not cancel: remove them
                key = my_key_agreement(sk_k, self.pk[i], self.p, self.g)
                r = np.random.RandomState(key % (2 ** 32)).randint(self.p, size=d).astype(np.int64)
                m_ik = (-r) % self.p if i > k else r  # mask client i added for pair (i, k)
                m_ik = r if i < k else (-r) % self.p
                s = (s - m_ik) % self.p
        return dequantize(s, self.scale, self.p)


class TA_Client:  # noqa: N801 (reference name)
    """Turbo-Aggregate participant (reference ``turboaggregate/TA_client.py:8-26``): local data handles plus the
    ``isdrop`` flag the protocol uses to simulate a client that drops out after uploading nothing; the
    server side recovers the masks of dropped clients in :meth:`TurboAggregateTrainer.server_aggregate`."""

    def __init__(self, local_training_data, local_test_data, local_sample_number, args, device, client_idx=0):
        self.local_training_data = local_training_data
        self.local_test_data = local_test_data
        self.local_sample_number = local_sample_number
        self.args, self.device, self.client_idx = args, device, client_idx
        import torch.nn as nn
        self.criterion = nn.CrossEntropyLoss()
        self.isdrop = False

    def set_dropout(self, isdrop):
        self.isdrop = bool(isdrop)

    def get_sample_number(self):
        return self.local_sample_number


def secure_round(trainer, clients, vectors, weights):
    """One Turbo-Aggregate round over ``TA_Client`` objects: every client that is not marked dropped uploads its
    masked, weighted update; the server removes the dropped clients' masks and returns the weighted sum."""
    uploads = {i: trainer.client_upload(i, vectors[i], weights[i]) for i, c in enumerate(clients) if not c.isdrop}
    dropped = [i for i, c in enumerate(clients) if c.isdrop]
    return trainer.server_aggregate(uploads, dropped=dropped)
