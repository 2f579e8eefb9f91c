"""N1 (config C3, BlockPruner 16 x 16 at 50 %): the MFMA count of a BRANCH-FREE per-row-group
compaction schedule (round-6 verdict item 3), on the masks `bench.py --prune block:16x16:0.5`
applies to D-38 (pruners/BlockPruner.py:139-241: blocks of 16 output x 16 input channels spanning
all 9 taps, `block_width *= unit_size` at :157-158, collapse_tensor off).

The schedule the verdict describes: a wave owns W output channels = W/16 row groups and, per K
step (one tap x 64 input channels = 4 channel blocks), pairs the live 16-channel blocks of each
row group into v_mfma_f32_16x16x32_bf16 MFMAs (K = 32 = two blocks), reading each lane's 16-B B
piece at its block's offset.  The accumulator a row group adds into must be a compile-time
register (acc[fm][fn]: AGPRs / VGPRs cannot be indexed at run time without a VALU move per
fragment), so a branch-free wave runs the SAME number of MFMAs M for every row group in a K step:
    M(wave, step) = max over its row groups r of ceil(live_r(step) / 2),   dense: 2.
Output channels may be permuted at pack time (the next layer's input channels with them) to put
row groups of similar live counts in one wave.  This prints, per pruned 3x3 layer and for W = 64
(conv_stag128's 64-channel waves) and W = 128 (the 128-channel waves of conv_stag and conv_w1,
which serve layer5-8), the ratio dense / sparse MFMA
count -- the speedup ceiling if the kernel stayed MFMA-bound and B-fragment selection were free --
  packed    channels in their natural order
  sorted    row blocks sorted by live count (the verdict's "sort output channels by live-block
            count"), then grouped consecutively
  greedy    a greedy grouping minimising sum over steps of M, plus a swap local search
  bound     for every step independently the best grouping of that step's counts (sorted, then
            consecutive groups): a lower bound on sum M valid for EVERY permutation, i.e. an upper
            bound on the speedup of any branch-free schedule of this form
and the FLOP-weighted network figures.

Operand delivery.  Dense, a wave's B fragment (one pixel group x one 32-channel block pair) feeds
all of its row groups; compacted, two row groups share a B fragment only if they pair the same
two blocks in that step, and the MFMA that consumes it names its B register at compile time --
so a branch-free wave reads one B fragment per MFMA.  The model at the end prices one K step of
the 8-wave staggered tile (wave = 128 channels x 64 pixels, 2 waves per SIMD) at the measured
rates: MFMA 16 cycles per v_mfma_f32_16x16x32_bf16 per SIMD, ds_read_b128 256 B/clk/CU
(MI355X_MICROARCH.md §LDS), the strip + weight DMA writes ~43 KB per step at ~128 B/clk.
python scripts/n1_branchfree_bound.py [seed]"""
import os
import sys
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-seg-model-compress_amd"))
sys.path.insert(0, ROOT)


def live_counts(w: np.ndarray) -> np.ndarray:
    """[row block][K step] -> number of live 16-channel blocks (0..4) in the step's 64 channels"""
    co, ci = w.shape[:2]
    live = np.abs(w).reshape(co // 16, 16, ci // 16, 16, -1).sum(axis=(1, 3, 4)) != 0   # [rb][cb16]
    return live.reshape(co // 16, ci // 64, 4).sum(axis=2)


def mfmas(cnt: np.ndarray, order, g: int) -> int:
    """sum over waves (g row groups, in `order`) and steps of max ceil(live / 2)"""
    need = (cnt[order] + 1) // 2                                          # [rb][step] in 0..2
    return int(need.reshape(-1, g, need.shape[1]).max(axis=1).sum())


def greedy(cnt, g, rng, iters=3000):
    R = cnt.shape[0]
    need = (cnt + 1) // 2
    left = list(range(R))
    order = []
    while left:
        seed = max(left, key=lambda r: need[r].sum())
        grp = [seed]
        left.remove(seed)
        cur = need[seed].copy()
        while len(grp) < g:
            best = min(left, key=lambda r: (np.maximum(cur, need[r]).sum() - cur.sum(), -need[r].sum()))
            grp.append(best)
            left.remove(best)
            cur = np.maximum(cur, need[best])
        order += grp
    order = np.array(order)
    best = mfmas(cnt, order, g)
    for _ in range(iters):
        a, b = rng.integers(0, R, 2)
        if a // g == b // g:
            continue
        order[[a, b]] = order[[b, a]]
        v = mfmas(cnt, order, g)
        if v <= best:
            best = v
        else:
            order[[a, b]] = order[[b, a]]
    return best


def bound(cnt, g) -> int:
    need = np.sort((cnt + 1) // 2, axis=0)[::-1]                          # per step, descending
    return int(need.reshape(-1, g, need.shape[1]).max(axis=1).sum())


def main():
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    import torch  # noqa: F401
    import bench
    args = types.SimpleNamespace(arch="drn_d_38", prune="block:16x16:0.5", precision="bf16", block_sparse=False)
    m, _ = bench.pruned_model(args, "cpu")
    rng = np.random.default_rng(seed)
    W = (64, 128)
    tot = {w: np.zeros(4) for w in W}
    dense_tot = {w: 0.0 for w in W}
    for name, p in m.state_dict().items():
        if not (name.startswith("layer.") and name.endswith(".weight") and p.dim() == 4 and p.shape[2] == 3):
            continue
        wt = p.float().numpy()
        co, ci = wt.shape[:2]
        if co % 64 or ci % 64:
            continue
        cnt = live_counts(wt)
        R, S = cnt.shape
        oh = {64: 256, 128: 128, 256: 128, 512: 128}.get(co, 128)          # D-38 rows at 1024 x 2048
        fl = 2.0 * co * ci * 9 * oh * 2 * oh                                # FLOP weight per frame
        hist = np.bincount(cnt.ravel(), minlength=5) / cnt.size
        line = [name, f"{co}x{ci}", "live/4 " + " ".join(f"{h:.2f}" for h in hist)]
        for w in W:
            g = min(w // 16, R)
            dense = 2 * (R // g) * S
            vals = [mfmas(cnt, np.arange(R), g),
                    mfmas(cnt, np.argsort(-cnt.sum(axis=1), kind="stable"), g),
                    greedy(cnt, g, rng), bound(cnt, g)]
            # FLOP-weighted: this layer's dense MFMA time x (sparse / dense)
            tot[w] += fl * np.array(vals) / dense
            dense_tot[w] += fl
            line.append(f"W{w}: " + " / ".join(f"{dense / v:.3f}x" for v in vals))
        print("  ".join(line), flush=True)
    # operand-delivery model, 8-wave staggered tile, one K step, per CU (greedy grouping's MFMAs)
    r = dense_tot[128] / tot[128][2]                  # dense / sparse MFMA count (greedy, W = 128)
    mf_dense = 64.0                                   # MFMAs per wave per K step (8 fm x 4 fn x 2 substeps)
    mf_sparse = mf_dense / r
    rd_dense = 2 * (8 + 4)                            # A + B fragment reads per wave per K step
    rd_sparse = mf_sparse + mf_sparse / 4             # one B read per MFMA + one A read per (fm, unit)
    dma = 43 * 1024 / 128.0
    t_mfma_d, t_mfma_s = 2 * mf_dense * 16, 2 * mf_sparse * 16
    t_lds_d, t_lds_s = 8 * rd_dense * 1024 / 256.0 + dma, 8 * rd_sparse * 1024 / 256.0 + dma
    print("\nOperand-delivery model (staggered tile, one K step per CU, greedy grouping):")
    print(f"  dense : {mf_dense:.1f} MFMAs / {rd_dense:.1f} fragment reads per wave -> MFMA {t_mfma_d:.0f} cyc, "
          f"LDS {t_lds_d:.0f} cyc -> bound {max(t_mfma_d, t_lds_d):.0f} cyc (MFMA)")
    print(f"  sparse: {mf_sparse:.1f} MFMAs / {rd_sparse:.1f} fragment reads per wave -> MFMA {t_mfma_s:.0f} cyc, "
          f"LDS {t_lds_s:.0f} cyc -> bound {max(t_mfma_s, t_lds_s):.0f} cyc "
          f"({'LDS' if t_lds_s > t_mfma_s else 'MFMA'}): {max(t_mfma_d, t_lds_d) / max(t_mfma_s, t_lds_s):.3f}x of dense")
    print("\nFLOP-weighted over the pruned 3x3 layers, dense / sparse MFMA count "
          "(packed / sorted / greedy / bound over all permutations):")
    for w in W:
        r = dense_tot[w] / tot[w]
        print(f"  W = {w:3d} channels per wave: " + " / ".join(f"{v:.3f}x" for v in r))


if __name__ == "__main__":
    main()
