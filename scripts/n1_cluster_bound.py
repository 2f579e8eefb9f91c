"""N1 (config C3, BlockPruner 16 x 16 at 50 %): how many K steps of a conv tile can be all-dead
once output channels (and, through the producer, input channels) are permuted to cluster dead
blocks -- the lever a block-sparse tile would need (pruners/BlockPruner.py:139-241, blocks of
16 output x 16 input channels spanning all 9 taps, collapse_tensor off).

A K step of the bf16 tiles covers one tap x 64 input channels = 4 channel blocks; a tile covers
T output channels = T / 16 row blocks.  The step is skippable for the tile iff all 4 x T/16
blocks are pruned.  Per pruned 3x3 layer of D-38 (the masks bench.py --prune block:16x16:0.5
applies) this prints, for T = 64 / 128 / 256:
  ident  fraction of all-dead (tile, K step) pairs in the packed order
  greedy the same after a greedy + local-search clustering of rows and columns (achievable)
  bound  an upper bound over EVERY row / column permutation: a row group of g = T/16 rows has at
         most floor(D*(g) / 4) dead K steps, D*(g) = the most columns any g rows are all dead on
         (exact by enumeration for g <= 8; D*(16) <= D*(8))
and the FLOP-weighted network figures with the Amdahl speedup 1 / (1 - f) a perfect skip gives.
python scripts/n1_cluster_bound.py [seed]"""
import os
import sys
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-seg-model-compress_amd"))
sys.path.insert(0, ROOT)


def block_dead(w: np.ndarray) -> np.ndarray:
    co, ci = w.shape[:2]
    b = np.abs(w).reshape(co // 16, 16, ci // 16, 16, -1).sum(axis=(1, 3, 4))
    return b == 0                                     # [row block][col block]


def pairs_dead(Z, rows, cols, g):
    """dead (row group, col group) pairs for row order `rows` (groups of g) and col order `cols`
    (groups of 4)"""
    R, C = Z.shape
    Zp = Z[np.ix_(rows, cols)]
    rg = Zp.reshape(R // g, g, C).all(axis=1)         # [row group][col]: dead for the whole group
    return int(rg.reshape(R // g, C // 4, 4).all(axis=2).sum())


def greedy(Z, g, rng, iters=4000):
    R, C = Z.shape
    left = list(range(R))
    rows = []
    while left:
        seed = max(left, key=lambda r: Z[r].sum())
        grp = [seed]
        left.remove(seed)
        common = Z[seed].copy()
        while len(grp) < g:
            best = max(left, key=lambda r: ((common & Z[r]).sum(), Z[r].sum()))
            grp.append(best)
            left.remove(best)
            common &= Z[best]
        rows += grp
    rg = Z[rows].reshape(R // g, g, C).all(axis=1)    # [group][col]
    leftc = list(range(C))
    cols = []
    while leftc:
        seed = max(leftc, key=lambda c: rg[:, c].sum())
        grp = [seed]
        leftc.remove(seed)
        common = rg[:, seed].copy()
        while len(grp) < 4:
            best = max(leftc, key=lambda c: ((common & rg[:, c]).sum(), rg[:, c].sum()))
            grp.append(best)
            leftc.remove(best)
            common &= rg[:, best]
        cols += grp
    best = pairs_dead(Z, rows, cols, g)
    rows, cols = np.array(rows), np.array(cols)
    for _ in range(iters):                            # local search: swap two rows or two columns
        if rng.random() < 0.5:
            a, b = rng.integers(0, R, 2)
            if a // g == b // g:
                continue
            rows[[a, b]] = rows[[b, a]]
            v = pairs_dead(Z, rows, cols, g)
            if v >= best:
                best = v
            else:
                rows[[a, b]] = rows[[b, a]]
        else:
            a, b = rng.integers(0, C, 2)
            if a // 4 == b // 4:
                continue
            cols[[a, b]] = cols[[b, a]]
            v = pairs_dead(Z, rows, cols, g)
            if v >= best:
                best = v
            else:
                cols[[a, b]] = cols[[b, a]]
    return best


def dstar(Z, g):
    """the most columns any g rows are all dead on (exact: depth-first over row subsets in
    increasing order, pruned once the running AND cannot beat the best found)"""
    R, C = Z.shape
    bits = [int("".join("1" if v else "0" for v in row), 2) for row in Z]
    best = [0]

    def dfs(start, depth, mask):
        if depth == g:
            best[0] = max(best[0], bin(mask).count("1"))
            return
        for r in range(start, R - (g - depth) + 1):
            m = mask & bits[r]
            if bin(m).count("1") > best[0]:
                dfs(r + 1, depth + 1, m)

    dfs(0, 0, (1 << C) - 1)
    return best[0]


def main():
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    import torch  # noqa: F401
    import bench
    args = types.SimpleNamespace(arch="drn_d_38", prune="block:16x16:0.5", precision="bf16", block_sparse=False)
    m, _ = bench.pruned_model(args, "cpu")
    rng = np.random.default_rng(seed)
    tot = {t: [0.0, 0.0, 0.0] for t in (64, 128, 256)}
    flops_all = 0.0
    rows_out = []
    for name, p in m.state_dict().items():
        if not (name.startswith("layer.") and name.endswith(".weight") and p.dim() == 4 and p.shape[2] == 3):
            continue
        w = p.float().numpy()
        co, ci = w.shape[:2]
        if co % 64 or ci % 64:
            continue
        Z = block_dead(w)
        if not Z.any():
            continue
        R, C = Z.shape
        oh = {64: 256, 128: 128, 256: 128, 512: 128}.get(co, 128)   # D-38 output rows at 1024 x 2048 / 8
        fl = 2.0 * co * ci * 9 * oh * 2 * oh                        # per frame (proportional weight)
        flops_all += fl
        line = [name, f"{co}x{ci}", f"{Z.mean():.3f}"]
        ds = {}
        for t in (64, 128, 256):
            g = min(t // 16, R)                       # a tile taller than the layer covers all of it
            n_pairs = (R // g) * (C // 4)
            ident = pairs_dead(Z, np.arange(R), np.arange(C), g) / n_pairs
            gr = greedy(Z, g, rng) / n_pairs
            gg = min(g, 8)
            if gg not in ds:
                ds[gg] = dstar(Z, gg) if R >= gg else 0
            bound = (ds[gg] // 4) / (C // 4)
            for k, v in enumerate((ident, gr, bound)):
                tot[t][k] += v * fl
            line.append(f"T{t}: {ident:.3f} / {gr:.3f} / {bound:.3f}")
        rows_out.append(line)
        print("  ".join(line), flush=True)
    print("\nFLOP-weighted over the pruned 3x3 layers (ident / greedy / bound) -> best-case speedup 1/(1-f):")
    for t in (64, 128, 256):
        f = [v / flops_all for v in tot[t]]
        print(f"  T = {t:3d} rows: {f[0]:.3f} / {f[1]:.3f} / {f[2]:.3f}  ->  "
              f"{1 / (1 - f[0]):.3f}x / {1 / (1 - f[1]):.3f}x / {1 / (1 - f[2]):.3f}x")


if __name__ == "__main__":
    main()
