"""Synthetic inputs shared by the development tools and bench.py."""
import numpy as np


def euclid(n, seed=1, dim=8):
    """Packed LT (reference order) of Euclidean distances between n random
    points in [0,1)^dim, rounded to 9 decimals like a Phylip matrix."""
    rng = np.random.default_rng(seed)
    pts = rng.random((n, dim))
    D = np.empty(n * (n - 1) // 2)
    for i in range(1, n):
        o = i * (i - 1) // 2
        D[o:o + i] = np.sqrt(((pts[:i] - pts[i]) ** 2).sum(1))
    return np.round(D * 1e9) / 1e9


def euclid_shard_dev(torch, n, rank, world, seed=4, dim=8, band=8, chunk_rows=512, dtype=None, cdist=False):
    """This rank's row bands (ccg_tree_shard_dev layout: bands of `band` rows
    dealt round-robin, owned rows back to back, row r = D(r, 0..r-1)) of the
    Euclidean distances between n points of U[0,1)^dim, computed on the GPU.
    Every rank draws the same points (CPU generator, fixed seed); computed in
    double, stored as `dtype` (default float64; float32 = `-p`).  cdist: the
    round-4 form (torch.cdist per chunk of rows), kept to reproduce that
    round's configs[3] matrix.  On this image's PyTorch-ROCm build
    torch.cdist gives wrong cells once a chunk has more than ~32k columns
    (tools/cdist_check.py, profiles/r06_generator_check.txt), so at n = 200k
    that form is not a Euclidean matrix."""
    g = torch.Generator().manual_seed(seed)
    pts = torch.rand((n, dim), generator=g, dtype=torch.float64).cuda()
    nb = (n + band - 1) // band
    mine = list(range(rank, nb, world))
    sizes = [sum(range(b * band, min(b * band + band, n))) for b in mine]
    out = torch.empty(max(sum(sizes), 1), dtype=dtype or torch.float64, device="cuda")
    per = max(1, chunk_rows // band)
    pos = 0
    for c0 in range(0, len(mine), per):
        bands = mine[c0:c0 + per]
        rows_h = [r for b in bands for r in range(b * band, min(b * band + band, n))]
        rows = torch.tensor(rows_h, device="cuda")
        rmax = rows_h[-1]
        if rmax == 0:
            continue
        # elementwise, one dimension at a time: every cell's value depends on
        # its two points only (torch.cdist's may depend on the batch's shape,
        # so the ranks of a world-8 run and the world-1 LT disagreed in the
        # last bit of some cells)
        if cdist:
            d = torch.cdist(pts[rows], pts[:rmax], compute_mode="donot_use_mm_for_euclid_dist")
        else:
            a, c = pts[rows][:, None, :], pts[:rmax][None, :, :]
            t = a[..., 0] - c[..., 0]
            s2 = t * t
            for k in range(1, dim):
                t = a[..., k] - c[..., k]
                s2 = s2 + t * t
            d = torch.sqrt(s2)
        # row-major: each row's prefix, rows in order (views concatenated: a
        # boolean-mask select of this size crashed torch inside a long process)
        vals = torch.cat([d[i, :r] for i, r in enumerate(rows_h) if r > 0])
        out[pos:pos + vals.numel()] = vals
        pos += vals.numel()
    assert pos == sum(sizes)
    return out


def clade_packed(n, L, clades, seed=3, every=10, flips=8):
    """A clade-structured packed alignment in the reference's layout, numpy
    only (the same bytes on the GPU box and in the build container): `clades`
    random root sequences, taxon t = root t % clades with each bit set to 1
    with p = 2^-flips xor-ed in (~0.8% of the 2-bit codes flipped at 8), as
    tools/config3.make_packed.  Returns (seqs n x W u64, W = L // 32 + 1
    words per taxon as cdist.c:290 allocates, positions past L zero;
    incs W u32: every `every`-th word excluded (the "N columns"), the tail
    past L cleared as initIncPos does, fsacmp.c:164)."""
    W = L // 32 + 1
    rng = np.random.default_rng(seed)
    roots = rng.integers(0, 2 ** 64, (clades, W), dtype=np.uint64, endpoint=False)
    seqs = np.empty((n, W), dtype=np.uint64)
    step = 4096
    for t0 in range(0, n, step):
        t1 = min(n, t0 + step)
        m = rng.integers(0, 2 ** 64, (t1 - t0, W), dtype=np.uint64, endpoint=False)
        for _ in range(flips - 1):
            m &= rng.integers(0, 2 ** 64, (t1 - t0, W), dtype=np.uint64, endpoint=False)
        seqs[t0:t1] = roots[np.arange(t0, t1) % clades] ^ m
    W32 = (L + 31) // 32
    seqs[:, W32:] = 0
    if L % 32:
        seqs[:, W32 - 1] &= np.uint64(((1 << (2 * (L % 32))) - 1) << (64 - 2 * (L % 32)))
    incs = np.full(W, 0xFFFFFFFF, dtype=np.uint32)
    if every:
        incs[::every] = 0
    incs[W32:] = 0
    if L % 32:
        incs[W32 - 1] &= np.uint32((0xFFFFFFFF << (32 - L % 32)) & 0xFFFFFFFF)
    return seqs, incs
