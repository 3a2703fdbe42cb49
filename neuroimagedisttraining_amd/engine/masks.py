"""Per-client sparse masks as bit rows, with per-layer ("segment") operations on device.

The reference keeps one ``{name: float tensor}`` mask dict per client and walks it in Python: DisPFL's fire / regrow
sorts every layer (``DisPFL/client.py:71-99``), SubAvg's ``fake_prune`` calls ``np.percentile`` per layer on the host
(``subavg/prune_func.py:9-30``), Hamming distances are Python loops (``DisPFL/slim_util.py:14-19``, scipy in
``subavg/prune_func.py:52-66``), and the masked average loops over clients (``subavg_api.py:123-139``).

Here every client's mask is one uint32 bit row over the flat parameter layout (``[R, W]`` int32 tensor, bit i of
word i >> 5 is parameter i — 1/32 of the float mask's bytes, read by the fused optimizer with the weights), and
every per-layer operation is one launch over all (client, layer) tiles:

* :meth:`MaskSpace.popcount` / :meth:`hamming` / :meth:`alive_count` — K17 / K18 counts per (client, layer);
* :meth:`MaskSpace.select` — K15 exact k-largest-key selection per (client, layer) (DisPFL fire / regrow);
* :meth:`MaskSpace.percentile_prune` — K16 SubAvg ``fake_prune`` with numpy's float32 ``percentile`` semantics;
* :func:`masked_rows_sum`, :func:`mix_rows`, :func:`pair_sqdist` — SubAvg averaging partials, gossip / neighbour
  mixing, and the parameter distances of FedFomo.

On a GPU the HIP kernels of ``csrc/kernels/sparse.hip`` run; on CPU (tests) the same semantics run in torch (ties
broken by the lowest index, exactly like the kernels and a stable sort).
"""
from __future__ import annotations

import numpy as np
import torch

from .. import ops

FIRE, REGROW_ABS, REGROW_RAND, ALIVE_MIN = 0, 1, 2, 3
TILE = 8192  # elements per work tile (a multiple of 32: tile boundaries inside a segment are word aligned)


def _hip(t):
    return t.device.type == "cuda"


def _st():
    return ops.stream()


def mask_words(P):
    """Words per bit row (16-byte aligned rows)."""
    return ((P + 31) // 32 + 3) // 4 * 4


# ------------------------------------------------------------------------------------------------ packing
def pack_bits(m):
    """``[R, P]`` bool/float (non-zero = 1) -> ``[R, W]`` int32 bit rows."""
    m = (m != 0)
    R, P = m.shape
    W = mask_words(P)
    pad = torch.zeros((R, W * 32), dtype=torch.bool, device=m.device)
    pad[:, :P] = m
    v = pad.view(R, W, 32).to(torch.int64) << torch.arange(32, device=m.device, dtype=torch.int64)
    s = v.sum(-1)
    return torch.where(s >= 2 ** 31, s - 2 ** 32, s).to(torch.int32)


def unpack_bits(bits, P, dtype=torch.float32):
    """``[R, W]`` int32 bit rows -> ``[R, P]`` 0/1 tensor (HIP: ``optim.hip`` ``k_unpack_bits`` for bool / fp32 — the
    torch form goes through an int64 [R, 32 W] temporary, 8 bytes per element, several passes)."""
    R, W = bits.shape
    if _hip(bits) and dtype in (torch.bool, torch.float32) and R and P:
        b = bits.contiguous()
        out = torch.empty((R, P), dtype=dtype, device=bits.device)
        ops.ext().unpack_bits_dev(b.data_ptr(), b.stride(0), R, P, int(dtype == torch.float32), out.data_ptr(), _st())
        return out
    b = (bits.to(torch.int64) & 0xffffffff).unsqueeze(-1) >> torch.arange(32, device=bits.device, dtype=torch.int64)
    return (b & 1).view(R, W * 32)[:, :P].to(dtype)


def masked_rows(dst, bits, src=None, P=None):
    """``dst[c, :P] = (src if given else dst[c, :P]) * mask_c`` with ``bits`` ``[C, W]`` (or ``[1, W]``: one mask for
    every row); ``dst`` ``[C, >= P]`` fp32 rows, ``src`` a ``[P]`` row.  HIP: one pass (``optim.hip`` ``k_masked_rows``)."""
    C = dst.shape[0]
    if P is None:
        P = src.numel() if src is not None else min(dst.shape[1], bits.shape[1] * 32)
    # the kernel reads 16-B row pieces and one bit row per dst row (or one shared row): anything else takes torch
    ok = (_hip(dst) and dst.dtype == torch.float32 and dst.stride(1) == 1 and dst.stride(0) % 4 == 0 and C
          and dst.data_ptr() % 16 == 0 and (src is None or (src.is_contiguous() and src.data_ptr() % 16 == 0))
          and bits.shape[0] in (1, C) and bits.shape[1] * 32 >= P)
    if ok:
        b = bits.contiguous()
        s = src.contiguous() if src is not None else None
        ops.ext().masked_rows(s.data_ptr() if s is not None else 0, b.data_ptr(), 0 if b.shape[0] == 1 else b.stride(0),
                              C, P, dst.stride(0), dst.data_ptr(), _st())
        return dst
    m = unpack_bits(bits, P)
    base = src.view(1, -1).expand(C, -1) if src is not None else dst[:, :P]
    dst[:, :P] = base * m
    return dst


# ------------------------------------------------------------------------------------------------ hash (regrow_rand)
def _mix_hash_np(seed, a, b):
    """numpy twin of ``mix_hash`` in sparse.hip (uint64 splitmix finaliser)."""
    with np.errstate(over="ignore"):
        a = np.asarray(a, dtype=np.uint64)
        b = np.asarray(b, dtype=np.uint64)
        z = np.uint64(seed) ^ (np.uint64(0x9e3779b97f4a7c15) * ((a << np.uint64(32)) ^ b))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
        z ^= z >> np.uint64(31)
        return (z >> np.uint64(32)).astype(np.uint64)


def _keys_torch(mode, v, bit, seed, cid, idx):
    """Selection keys (int64, larger first, 0 = not a candidate) — the torch twin of ``sel_key``."""
    if mode == REGROW_RAND:
        h = torch.from_numpy((_mix_hash_np(seed, cid, idx.cpu().numpy()) | np.uint64(1)).astype(np.int64))
        return torch.where(bit, torch.zeros_like(h), h.to(bit.device))
    a = (v.float().contiguous().view(torch.int32).to(torch.int64) & 0x7fffffff)
    if mode == FIRE:
        return torch.where(bit, 0xffffffff - a, torch.zeros_like(a))
    if mode == REGROW_ABS:
        return torch.where(bit, torch.zeros_like(a), a + 1)
    return torch.where(bit & (a != 0), 0xffffffff - a, torch.zeros_like(a))  # ALIVE_MIN


class MaskSpace:
    """Segments (per-parameter ranges of a flat layout) and the tile tables of per-(row, segment) launches."""

    def __init__(self, layout, names=None):
        self.layout = layout
        self.P = layout.total
        self.W = mask_words(self.P)
        names = list(layout.names) if names is None else list(names)
        self.names = names
        idx = [layout.names.index(n) for n in names]
        self.seg = np.array([[layout.offsets[i], layout.offsets[i] + layout.numel(i)] for i in idx], dtype=np.int64)
        self.S = len(names)
        self.seg_len = self.seg[:, 1] - self.seg[:, 0]
        self._tiles = {}

    def seg_mask(self):
        """Boolean [P]: covered by some segment."""
        m = torch.zeros(self.P, dtype=torch.bool)
        for b, e in self.seg:
            m[b:e] = True
        return m

    def tiles(self, R, device):
        key = (R, str(device))
        if key not in self._tiles:
            rows = []
            for s, (b, e) in enumerate(self.seg):
                cuts = [int(b)] + list(range((int(b) // TILE + 1) * TILE, int(e), TILE))
                for j, c in enumerate(cuts):
                    rows.append((s, c, cuts[j + 1] if j + 1 < len(cuts) else int(e), j))
            per = np.array([(s, c0, c1) for s, c0, c1, _ in rows], dtype=np.int64).reshape(-1, 3)
            first_in_seg = np.array([j for *_, j in rows], dtype=np.int64)
            T0 = len(per)
            tiles = np.zeros((R * T0, 4), dtype=np.int32)
            first = np.zeros(R * T0, dtype=np.int32)
            for r in range(R):
                sl = slice(r * T0, (r + 1) * T0)
                tiles[sl, 0] = r
                tiles[sl, 1] = per[:, 0]
                tiles[sl, 2] = per[:, 1]
                tiles[sl, 3] = per[:, 2]
                first[sl] = np.arange(r * T0, (r + 1) * T0) - first_in_seg
            self._tiles[key] = (torch.from_numpy(tiles).to(device), torch.from_numpy(first).to(device), R * T0)
        return self._tiles[key]

    # -------------------------------------------------------------------------------------------- counts
    def _count(self, mode, A, Bm=None, v=None):
        R = A.shape[0]
        if _hip(A):
            tiles, _, nt = self.tiles(R, A.device)
            out = torch.zeros((R, self.S), dtype=torch.int32, device=A.device)
            ops.ext().seg_count(tiles.data_ptr(), nt, A.data_ptr(), Bm.data_ptr() if Bm is not None else 0,
                                A.stride(0), v.data_ptr() if v is not None else 0, v.stride(0) if v is not None else 0,
                                mode, self.S, out.data_ptr(), _st())
            return out.to(torch.int64)
        a = unpack_bits(A, self.P, torch.bool)
        if mode == 1:
            a = a ^ unpack_bits(Bm, self.P, torch.bool)
        elif mode == 2:
            a = a & (v[:, :self.P] != 0)
        return torch.stack([a[:, b:e].sum(1) for b, e in self.seg], 1).to(torch.int64)

    def popcount(self, bits):
        return self._count(0, bits)

    def hamming(self, a, b):
        return self._count(1, a, b)

    def alive_count(self, bits, v):
        """Entries with mask 1 and value != 0 (SubAvg's ``alive``) per (row, segment)."""
        return self._count(2, bits, v=v)

    # -------------------------------------------------------------------------------------------- selection
    def select(self, mode, v, bits, k, cids=None, seed=0, query_only=False):
        """Per (row, segment): take the ``k[r, s]`` largest keys (see sparse.hip) among the candidates and clear
        (FIRE) or set (REGROW_*) their bits in place.  ``query_only`` returns the k-th key's value instead: for
        ALIVE_MIN the k-th smallest alive |v| ([R, S] float32, NaN where k == 0).  ``k`` must not exceed the
        number of candidates of its segment."""
        R = bits.shape[0]
        k = k.to(torch.int64)
        assert k.shape == (R, self.S) and bits.shape[1] >= (self.P + 31) // 32 and bits.stride(1) == 1
        assert v is None or (v.shape[0] >= R and v.shape[1] >= self.P and v.stride(1) == 1)
        if _hip(bits):
            dev = bits.device
            tiles, first, nt = self.tiles(R, dev)
            nseg = R * self.S
            state = torch.zeros((nseg, 4), dtype=torch.int32, device=dev)
            state[:, 2] = k.reshape(-1).to(torch.int32)
            hist = torch.zeros((nseg, 256), dtype=torch.int32, device=dev)
            ties = torch.zeros(max(1, nt), dtype=torch.int32, device=dev)
            ct = None
            if cids is not None:
                ct = torch.as_tensor(np.asarray(cids, dtype=np.int32)).to(dev)
            vp = v.data_ptr() if v is not None else 0
            ld = v.stride(0) if v is not None else 0
            ops.ext().seg_select(tiles.data_ptr(), first.data_ptr(), nt, vp, ld, bits.data_ptr(), bits.stride(0),
                                 ct.data_ptr() if ct is not None else 0, int(seed) & ((1 << 64) - 1), R, self.S, mode,
                                 state.data_ptr(), hist.data_ptr(), ties.data_ptr(), int(query_only), _st())
            if query_only:
                T = state[:, 3].view(R, self.S).to(torch.int64) & 0xffffffff
                val = (0xffffffff - T).to(torch.int32).view(torch.float32)
                return torch.where(k > 0, val, torch.full_like(val, float("nan")))
            return None
        return self._select_torch(mode, v, bits, k, cids, seed, query_only)

    def _select_torch(self, mode, v, bits, k, cids, seed, query_only):
        R = bits.shape[0]
        m = unpack_bits(bits, self.P, torch.bool)
        out = torch.full((R, self.S), float("nan"))
        for r in range(R):
            cid = int(cids[r]) if cids is not None else r
            for s, (b, e) in enumerate(self.seg):
                kk = int(k[r, s])
                if kk <= 0:
                    continue
                idx = torch.arange(int(b), int(e))
                vv = v[r, b:e] if v is not None else None
                key = _keys_torch(mode, vv, m[r, b:e], seed, cid, idx)
                order = torch.sort(key, descending=True, stable=True).indices[:kk]
                if query_only:
                    out[r, s] = float(torch.tensor([int(0xffffffff - int(key[order[-1]]))],
                                                   dtype=torch.int64).to(torch.int32).view(torch.float32))
                    continue
                m[r, b + order] = mode != FIRE
        if query_only:
            return out.to(bits.device)
        bits.copy_(pack_bits(m))
        return None

    # -------------------------------------------------------------------------------------------- SubAvg prune
    def percentile_prune(self, v, bits, ratio, prune_names):
        """SubAvg ``fake_prune``: per (row, prunable segment) thr = numpy.percentile(|alive|, 100 * ratio) computed
        with numpy's float32 arithmetic, new mask = old mask & (|w| >= thr).  Returns new bit rows."""
        R = bits.shape[0]
        prune = np.array([1 if n in set(prune_names) else 0 for n in self.names], dtype=np.int32)
        n = self.alive_count(bits, v).cpu().numpy()
        q = np.asanyarray(np.true_divide(ratio * 100, np.float32(100)))
        lo = np.zeros((R, self.S), dtype=np.int64)
        hi = np.zeros((R, self.S), dtype=np.int64)
        gam = np.zeros((R, self.S), dtype=np.float32)
        for r in range(R):
            for s in range(self.S):
                cnt = int(n[r, s])
                if not prune[s] or cnt == 0:
                    continue
                vi = cnt * q + (1 + q * (1 - 1 - 1)) - 1  # numpy _compute_virtual_index (linear), float32
                p = np.asanyarray(np.floor(vi))
                if vi >= cnt - 1:
                    a = b = cnt - 1
                elif vi < 0:
                    a = b = 0
                else:
                    a = int(p)
                    b = a + 1
                lo[r, s], hi[r, s] = a + 1, b + 1
                gam[r, s] = np.asanyarray(vi - np.asanyarray(p).astype(np.intp), dtype=np.float32)
        dev = bits.device
        va = self.select(ALIVE_MIN, v, bits, torch.from_numpy(lo).to(dev), query_only=True).cpu().numpy()
        vb = self.select(ALIVE_MIN, v, bits, torch.from_numpy(hi).to(dev), query_only=True).cpu().numpy()
        thr = np.full((R, self.S), np.nan, dtype=np.float32)
        for r in range(R):
            for s in range(self.S):
                if not prune[s] or n[r, s] == 0:
                    continue
                a, b, t = np.float32(va[r, s]), np.float32(vb[r, s]), np.asanyarray(gam[r, s])
                d = np.subtract(b, a)
                val = np.add(a, d * t)
                if t >= 0.5:
                    val = np.subtract(b, d * (1 - t))
                thr[r, s] = np.float32(val)
        out = bits.clone()
        thr_t = torch.from_numpy(thr).to(dev)
        if _hip(bits):
            tiles, _, nt = self.tiles(R, dev)
            pr = torch.from_numpy(prune).to(dev)
            ops.ext().seg_prune(tiles.data_ptr(), nt, v.data_ptr(), v.stride(0), out.data_ptr(), out.stride(0),
                                thr_t.data_ptr(), pr.data_ptr(), self.S, _st())
            return out
        m = unpack_bits(bits, self.P, torch.bool)
        for s, (b, e) in enumerate(self.seg):
            if prune[s]:
                m[:, b:e] &= ~(v[:, b:e].abs() < thr_t[:, s:s + 1])
        return pack_bits(m)


# ------------------------------------------------------------------------------------------------ row ops
def masked_rows_sum(rows, n, bits, sum_, cnt):
    """sum_[p] += sum_r rows[r, p]; cnt[p] += sum_r bit(r, p) (bits None: every row counts)."""
    R = rows.shape[0]
    if R == 0 or n == 0:  # n = 0: models without buffers (GroupNorm ResNets)
        return
    if _hip(rows):
        assert rows.stride(1) == 1 and rows.shape[1] >= n and sum_.numel() >= n and cnt.numel() >= n
        assert bits is None or (bits.shape[0] == R and bits.shape[1] * 32 >= n and bits.stride(1) == 1)
        ops.ext().masked_rows_sum(rows.data_ptr(), rows.stride(0), bits.data_ptr() if bits is not None else 0,
                                  bits.stride(0) if bits is not None else 0, R, n, sum_.data_ptr(), cnt.data_ptr(),
                                  _st())
        return
    sum_ += rows[:, :n].sum(0)
    if bits is None:
        cnt += R
    else:
        cnt += unpack_bits(bits, n).sum(0)


def masked_mean_rows(plan, n):
    """``plan``: list of ``(dst_row, own_bits_row, [(src_row, src_bits_row), ...])``: dst[p] = own(p) * mean of the
    src rows whose bit p is set (0 where none is) — DisPFL's masked neighbour average.  fp32 rows of length >= n,
    uint32 bit rows; dst must not alias a source.  One launch for every output row."""
    plan = [p for p in plan if p[2]]
    if not plan or n == 0:
        return
    d0 = plan[0][0]
    if _hip(d0):
        assert all(d.data_ptr() % 16 == 0 and all(t.data_ptr() % 16 == 0 for t, _ in terms) for d, _, terms in plan), \
            "masked_mean_rows: rows must be 16-byte aligned"
        src, sb, rp, dst, own = [], [], [0], [], []
        for d, ob, terms in plan:
            dst.append(d.data_ptr())
            own.append(ob.data_ptr())
            for t, b in terms:
                src.append(t.data_ptr())
                sb.append(b.data_ptr())
            rp.append(len(src))
        dev = d0.device
        # named: the tables must stay referenced until the launch is enqueued (a temporary's block could be
        # handed to the next table's copy first)
        t_src, t_sb = torch.tensor(src, dtype=torch.int64).to(dev), torch.tensor(sb, dtype=torch.int64).to(dev)
        t_rp, t_dst = torch.tensor(rp, dtype=torch.int32).to(dev), torch.tensor(dst, dtype=torch.int64).to(dev)
        t_own = torch.tensor(own, dtype=torch.int64).to(dev)
        ops.ext().masked_mean_rows(t_src.data_ptr(), t_sb.data_ptr(), t_rp.data_ptr(), t_dst.data_ptr(),
                                   t_own.data_ptr(), len(plan), n, _st())
        return
    for d, ob, terms in plan:
        num = torch.zeros(n, dtype=torch.float32, device=d.device)
        cnt = torch.zeros(n, dtype=torch.float32, device=d.device)
        for t, b in terms:
            m = unpack_bits(b.view(1, -1), n, torch.bool)[0]
            num += torch.where(m, t[:n], torch.zeros_like(num))
            cnt += m.float()
        o = unpack_bits(ob.view(1, -1), n, torch.bool)[0]
        d[:n] = torch.where((cnt > 0) & o, num / cnt.clamp_min(1), torch.zeros_like(num))


def mix_rows(plan, n):
    """``plan``: list of ``(dst_row, [(src_row, weight), ...])`` 1-D fp32 tensors of length >= n; dst rows must not
    alias sources.  One launch for every output row."""
    if not plan or n == 0:
        return
    dev = plan[0][0].device
    if _hip(plan[0][0]):
        assert all(d.data_ptr() % 16 == 0 and all(t.data_ptr() % 16 == 0 for t, _ in terms) for d, terms in plan), \
            "mix_rows: rows must be 16-byte aligned"
        src, wts, rp, dst = [], [], [0], []
        for d, terms in plan:
            dst.append(d.data_ptr())
            for s, w in terms:
                src.append(s.data_ptr())
                wts.append(float(w))
            rp.append(len(src))
        t_src = torch.tensor(src, dtype=torch.int64).to(dev)
        t_w = torch.tensor(wts, dtype=torch.float32).to(dev)
        t_rp = torch.tensor(rp, dtype=torch.int32).to(dev)
        t_dst = torch.tensor(dst, dtype=torch.int64).to(dev)
        ops.ext().mix_rows(t_src.data_ptr(), t_w.data_ptr(), t_rp.data_ptr(), t_dst.data_ptr(), len(plan), n, _st())
        return
    for d, terms in plan:
        acc = torch.zeros(n, dtype=torch.float32, device=dev)
        for s, w in terms:
            acc.add_(s[:n], alpha=float(w))
        d[:n].copy_(acc)


def pair_sqdist(pairs, n):
    """``pairs``: list of ``(a_row, b_row)`` -> float64 tensor of sum((a - b)^2) over the first n entries."""
    if not pairs:
        return torch.zeros(0, dtype=torch.float64)
    dev = pairs[0][0].device
    if n == 0:
        return torch.zeros(len(pairs), dtype=torch.float64, device=dev)
    if _hip(pairs[0][0]):
        assert all(a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0 for a, b in pairs), "pair_sqdist: alignment"
        m = ops.ext()
        nb = m.pair_sqdist_nblk(n)
        part = torch.empty((len(pairs), nb), dtype=torch.float32, device=dev)
        pa = torch.tensor([a.data_ptr() for a, _ in pairs], dtype=torch.int64).to(dev)
        pb = torch.tensor([b.data_ptr() for _, b in pairs], dtype=torch.int64).to(dev)
        m.pair_sqdist(pa.data_ptr(), pb.data_ptr(), len(pairs), n, part.data_ptr(), _st())
        return part.double().sum(1)
    return torch.stack([((a[:n].double() - b[:n].double()) ** 2).sum() for a, b in pairs])
