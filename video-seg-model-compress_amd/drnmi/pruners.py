"""Pruner API drop-in: Block / RMB / SRMB-Rep mask generators + HIP mask-apply.

Reference interface (kept name-for-name):
  Pruner(config_fp, on_gpu=True)          pruners/Pruner.py:6-15
  .mask_dict  OrderedDict[key -> fp32 mask tensor, weight-shaped]
  .layer_configs = parse_config_file(fp)  per-subclass JSON schema
  .generate_masks(model, is_static=..., verbose=False)
  .apply_masks(model)                     pruners/Pruner.py:17-20  (w *= mask, in place)
  .print_stats()                          pruners/Pruner.py:22-27
  BlockPruner                             pruners/BlockPruner.py:76-432
  RmbPruner                               pruners/RmbPruner.py:78-378
  SRMBRepMasker                           pruners/SRMBRepMasker.py:51-383
  make_pruner(config_fp)                  semantic_seg.py:822-847 (pruner_type dispatch)

Mask generation is one-off host work (numpy) and reproduces the reference masks
bit-for-bit, including the np.random call sequence of the random patterns, so a
seeded run gives the same masks (tests/test_pruners_golden.py).  Where the
reference loops per block in Python, the block sums are computed for all blocks at
once with the same float32 reduction order.

apply_masks is the hot step (called after every optimizer step, semantic_seg.py:
213-214): ONE multi-tensor HIP launch over all masked layers (drnmi_mask_apply_*),
in place on the parameter storage, bit-identical to `w *= mask`.

Deliberate deviations (documented, not silent):
  * BlockPruner sub-matrix mode raises ValueError when sub_rows/sub_cols do not
    divide the matrix (the reference recurses without end there).
  * RmbPruner.generate_masks accepts and ignores is_static (reference signature lacks
    it, so semantic_seg.py:849 raises TypeError).
  * apply_masks resolves a 'module.' prefix (DataParallel/DDP) and the seg_video
    'base.' prefix; the reference raises KeyError.
"""
from __future__ import annotations

import collections
import ctypes
import itertools
import json

import numpy as np
import torch

from . import _lib


# ============================================================================ base
class Pruner:
    """Super class: owns mask_dict and the fused apply."""

    def __init__(self, config_fp, on_gpu=True):
        self.config_fp = config_fp
        self.on_gpu = on_gpu
        self.mask_dict = collections.OrderedDict()
        self.layer_configs = self.parse_config_file(config_fp)
        self._bits_cache = {}
        self._binary_cache = {}
        self._factors = {}           # layer -> compact mask factors (SRMBRepMasker period tiles)

    # -- subclasses implement
    def parse_config_file(self, config_fp):  # pragma: no cover - abstract
        raise NotImplementedError

    def _store(self, layer, mask: np.ndarray):
        t = torch.from_numpy(np.ascontiguousarray(mask))
        self.mask_dict[layer] = t.cuda() if self.on_gpu else t
        self._bits_cache.pop(layer, None)
        self._factors.pop(layer, None)

    # -- the hot step
    def apply_masks(self, model, use_bits: bool = True):
        """In-place `w *= mask` for every masked layer, one HIP launch for all of them."""
        if not self.mask_dict:
            return
        params = _resolve_tensors(model, list(self.mask_dict))
        if use_bits and not all(self._is_binary(layer) for layer in params):
            use_bits = False      # a non-0/1 mask: w *= mask with the fp32 mask kernel (Pruner.py:20)
        ws, ms, ns = [], [], []
        for layer, w in params.items():
            m = self.mask_dict[layer]
            if not w.is_cuda:
                raise RuntimeError("Pruner.apply_masks runs on the HIP kernel: model must be on a ROCm "
                                   "device (no CPU fallback by design)")
            if w.dtype != torch.float32 or not w.is_contiguous():
                raise RuntimeError(f"{layer}: expected contiguous fp32 weight")
            if m.shape != w.shape:
                raise RuntimeError(f"{layer}: mask shape {tuple(m.shape)} != weight {tuple(w.shape)}")
            ws.append(w)
            ns.append(w.numel())
            if use_bits:
                ms.append(self._mask_bits(layer, w.device))
            else:
                mm = m if (m.is_cuda and m.device == w.device and m.dtype == torch.float32) else \
                    m.to(w.device, torch.float32)
                ms.append(mm.contiguous())
        lib = _lib.load()
        n = len(ws)
        wp = (ctypes.c_void_p * n)(*[w.data_ptr() for w in ws])
        mp = (ctypes.c_void_p * n)(*[m.data_ptr() for m in ms])
        npn = (ctypes.c_int64 * n)(*ns)
        stream = ctypes.c_void_p(_lib.stream_ptr(ws[0].device))
        fn = lib.drnmi_mask_apply_bits_f32 if use_bits else lib.drnmi_mask_apply_f32
        _lib.check(fn(n, wp, mp, npn, stream), "mask_apply")
        for w in ws:        # in-place write through the C-ABI: bump the version counters
            torch.autograd.graph.increment_version(w)   # (DRNSeg repacks on change)

    def _is_binary(self, layer) -> bool:
        """True when mask_dict[layer] holds only 0 and 1 (what the 1-bit formats can represent)."""
        m = self.mask_dict[layer]
        key = (m.data_ptr(), m._version)
        hit = self._binary_cache.get(layer)
        if hit is None or hit[0] != key:
            hit = (key, bool(((m == 0) | (m == 1)).all().item()))
            self._binary_cache[layer] = hit
        return hit[1]

    def _mask_bits(self, layer, device):
        """Bit-packed copy of mask_dict[layer] (bit i of word i/32), cached per mask tensor.
        Raises ValueError for a mask that is not 0/1 valued (it would be silently binarised)."""
        m = self.mask_dict[layer]
        key = (m.data_ptr(), m._version, str(device))
        hit = self._bits_cache.get(layer)
        if hit is not None and hit[0] == key:
            return hit[1]
        if not self._is_binary(layer):
            raise ValueError(f"{layer}: mask is not 0/1 valued; the 1-bit mask path cannot hold it")
        words = _pack_bits((m.detach().reshape(-1) != 0).cpu().numpy())
        bits = torch.from_numpy(words.view(np.int32).copy()).to(device)
        self._bits_cache[layer] = (key, bits)
        return bits

    # -- compact on-disk masks (the reference never persists masks,
    #    semantic_seg.py:1085-1092, so an SRMB run cannot be resumed with the same masks)
    def save_masks(self, path):
        """Write mask_dict to an .npz in the most compact exact form per layer:
          * SRMBRepMasker masks still equal to their generated factors: the factors -- OB and the
            period tile P as bits plus the block sizes (kind 1), or the non-repetitive block
            pattern OCP (kind 2); the whole mask is their kron (SRMBRepMasker.py:337-383).  All
            factor bits of all layers share one word array, so a D-22 SRMB mask set is ~2 KB;
          * any other mask: 1 bit per weight in the apply kernel's word layout (kind 0).
        Masks must be 0/1 valued (every reference pruner stores 0./1. floats); anything else
        raises ValueError rather than being silently binarised."""
        layers = list(self.mask_dict)
        arrays = {"format": np.array([MASK_FORMAT_VERSION], dtype=np.int64),
                  "layers": np.array(layers, dtype=np.str_)}
        shapes = np.ones((len(layers), 4), dtype=np.int64)
        ndims = np.zeros(len(layers), dtype=np.int64)
        dtypes = []
        meta = np.zeros((len(layers), 12), dtype=np.int64)   # kind, ib(2), cb(2), A(2), B(2), offA, offB, 0
        fwords, off = [], 0
        for i, (layer, m) in enumerate(self.mask_dict.items()):
            a = m.detach().cpu().numpy()
            nz = a != 0
            if not np.array_equal(a[nz], np.ones(int(nz.sum()), dtype=a.dtype)):
                raise ValueError(f"{layer}: mask is not 0/1 valued; the bit format cannot hold it")
            if a.ndim > 4:
                raise ValueError(f"{layer}: masks of more than 4 dimensions are not supported")
            ndims[i] = a.ndim
            shapes[i, :a.ndim] = a.shape
            dtypes.append(str(a.dtype))
            fac = self._factors.get(layer)
            if fac is not None and np.array_equal(SRMBRepMasker.expand_factors(fac) != 0, nz):
                grids = [fac["ob"], fac["p"]] if fac["rep"] else [fac["ocp"]]
                meta[i, 0] = 1 if fac["rep"] else 2
                meta[i, 1:3] = fac["ib"]
                if fac["rep"]:
                    meta[i, 3:5] = fac["cb"]
                for j, g in enumerate(grids):
                    g = np.asarray(g)
                    w = _pack_bits(g.reshape(-1) != 0)
                    meta[i, 5 + 2 * j:7 + 2 * j] = g.shape
                    meta[i, 9 + j] = off
                    fwords.append(w)
                    off += w.size
                continue
            arrays[f"bits{i}"] = _pack_bits(nz.reshape(-1))
        arrays.update(shapes=shapes, ndims=ndims, dtypes=np.array(dtypes, dtype=np.str_), meta=meta,
                      fwords=np.concatenate(fwords) if fwords else np.zeros(0, dtype=np.uint32))
        with open(path, "wb") as f:
            np.savez_compressed(f, **arrays)

    def load_masks(self, path):
        """Restore mask_dict from save_masks() output (format 1: bits only, or 2); seeds the bit
        cache so the next apply_masks uploads no fp32 mask at all."""
        with np.load(path, allow_pickle=False) as z:
            version = int(z["format"][0])
            if version not in (1, MASK_FORMAT_VERSION):
                raise ValueError(f"{path}: mask format {version} is not 1..{MASK_FORMAT_VERSION}")
            self.mask_dict = collections.OrderedDict()
            self._bits_cache = {}
            self._binary_cache = {}
            self._factors = {}
            fwords = z["fwords"] if version >= 2 else None
            for i, layer in enumerate(z["layers"].tolist()):
                if version >= 2:
                    shape = tuple(int(v) for v in z["shapes"][i, :int(z["ndims"][i])])
                    dt = str(z["dtypes"][i])
                    meta = [int(v) for v in z["meta"][i]]
                else:
                    shape = tuple(int(v) for v in z[f"shape{i}"])
                    dt = str(z[f"dtype{i}"][0])
                    meta = [0] * 12
                n = int(np.prod(shape))
                kind = meta[0]
                if kind in (1, 2):
                    def grid(j):
                        shp = (meta[5 + 2 * j], meta[6 + 2 * j])
                        cnt = shp[0] * shp[1]
                        w = fwords[meta[9 + j]:meta[9 + j] + (cnt + 31) // 32]
                        if w.size != (cnt + 31) // 32:
                            raise ValueError(f"{path}: {layer}: truncated factor words")
                        return _unpack_bits(w, cnt).reshape(shp).astype(np.float64)
                    fac = {"shape": shape, "dtype": dt, "ib": (meta[1], meta[2]), "rep": kind == 1}
                    if kind == 1:
                        fac.update(ob=grid(0), p=grid(1), cb=(meta[3], meta[4]))
                    else:
                        fac.update(ocp=grid(0).astype(dt))
                    mask = SRMBRepMasker.expand_factors(fac)
                    if mask.size != n:
                        raise ValueError(f"{path}: {layer}: factors expand to {mask.size} weights, not {n}")
                    self._store(layer, mask.astype(dt))
                    self._factors[layer] = fac
                    words = _pack_bits(mask.reshape(-1) != 0)
                elif kind == 0:
                    words = z[f"bits{i}"]
                    if words.dtype != np.uint32 or words.size != (n + 31) // 32:
                        raise ValueError(f"{path}: {layer}: {words.size} words for {n} weights")
                    mask = _unpack_bits(words, n).reshape(shape).astype(dt)
                    self._store(layer, mask)
                else:
                    raise ValueError(f"{path}: {layer}: unknown mask kind {kind}")
                if self.on_gpu:
                    m = self.mask_dict[layer]
                    self._bits_cache[layer] = ((m.data_ptr(), m._version, str(m.device)),
                                               torch.from_numpy(words.view(np.int32).copy()).to(m.device))
        return self

    def print_stats(self):
        for layer in self.mask_dict:
            mask_np = self.mask_dict[layer].cpu().numpy()
            sp = 1.0 - np.count_nonzero(mask_np) / mask_np.size
            print(layer, "sparsity = {}".format(sp * 100))


MASK_FORMAT_VERSION = 2   # 1: bits only; 2: + SRMB factor (period-tile) layers


def _pack_bits(flat: np.ndarray) -> np.ndarray:
    """bool[n] -> uint32[ceil(n/32)], weight i is bit (i % 32) of word i // 32 (LSB first) —
    the layout drnmi_mask_apply_bits_f32 reads."""
    flat = np.asarray(flat, dtype=bool)
    pad = (-flat.size) % 32
    if pad:
        flat = np.concatenate([flat, np.zeros(pad, dtype=bool)])
    return np.packbits(flat.reshape(-1, 32), axis=1, bitorder="little").view("<u4").astype(np.uint32).reshape(-1)


def _unpack_bits(words: np.ndarray, n: int) -> np.ndarray:
    b = np.unpackbits(np.ascontiguousarray(words, dtype="<u4").view(np.uint8), bitorder="little")
    return b[:n].astype(bool)


def _resolve_tensors(model, layers):
    sd = model.state_dict()
    out = collections.OrderedDict()
    for layer in layers:
        for cand in (layer, "module." + layer, layer.replace("layer.", "base.", 1),
                     layer[len("module."):] if layer.startswith("module.") else None):
            if cand is not None and cand in sd:
                out[layer] = sd[cand]
                break
        else:
            raise KeyError(layer)
    return out


def _load_configs(config_fp):
    with open(config_fp) as f:
        return json.load(f)


def make_pruner(config_fp, on_gpu=True):
    """JSON pruner_type dispatch (semantic_seg.py:822-847)."""
    kind = _load_configs(config_fp)["pruner_type"]
    table = {"block": BlockPruner, "rmb": RmbPruner, "srmbrep": SRMBRepMasker}
    if kind not in table:
        raise NotImplementedError(f"pruner_type {kind!r}: hb/rmcdb/grouping mask generators are out of "
                                  "scope (their masks still apply through Pruner.apply_masks)")
    return table[kind](config_fp, on_gpu)


def _block_abs_sums(mat: np.ndarray, bh: int, bw: int) -> np.ndarray:
    """np.sum(np.abs(block)) for every (bh x bw) block of a 2-D matrix, ragged edge blocks
    included, with the same float32 reduction as the reference's per-block np.sum of a
    contiguous copy (BlockPruner.py:183-190, RmbPruner.py:150-152)."""
    rows, cols = mat.shape
    nrb, ncb = -(-rows // bh), -(-cols // bw)
    a = np.abs(mat)
    out = np.zeros((nrb, ncb), dtype=mat.dtype)
    fr, fc = rows // bh, cols // bw
    if fr and fc:
        core = a[:fr * bh, :fc * bw].reshape(fr, bh, fc, bw).transpose(0, 2, 1, 3)
        out[:fr, :fc] = np.ascontiguousarray(core).reshape(fr, fc, bh * bw).sum(axis=2)
    for rb in range(nrb):              # ragged edges: exact per-block copies
        for cb in range(ncb):
            if rb < fr and cb < fc:
                continue
            blk = a[rb * bh:min(rows, (rb + 1) * bh), cb * bw:min(cols, (cb + 1) * bw)]
            out[rb, cb] = np.sum(np.ascontiguousarray(blk))
    return out


def _expand_blocks(keep: np.ndarray, bh: int, bw: int, rows: int, cols: int, dtype) -> np.ndarray:
    return np.kron(keep.astype(dtype), np.ones((bh, bw), dtype=dtype))[:rows, :cols]


# ============================================================================ BlockPruner
class BlockPrunerConfig:
    def __init__(self, sparsity, block_height, block_width, sub_rows, sub_cols, collapse_tensor):
        self.sparsity = sparsity
        self.block_height = block_height
        self.block_width = block_width
        self.sub_rows = sub_rows
        self.sub_cols = sub_cols
        self.collapse_tensor = collapse_tensor

    def __str__(self):
        return "{} {} {}".format(self.block_height, self.block_width, self.sparsity)


class BlockMatrix:
    """BSR container (BlockPruner.py:55-74)."""

    def __init__(self, rows, cols, bh, bw, values, indices, rowBlockPtr):
        self.rows, self.cols, self.bh, self.bw = rows, cols, bh, bw
        self.values, self.indices, self.rowBlockPtr = values, indices, rowBlockPtr


class BlockPruner(Pruner):
    def parse_config_file(self, config_fp):
        cfg = collections.OrderedDict()
        for ls in _load_configs(config_fp)["configs"]:
            c = BlockPruner.generate_block_pruner_config(ls)
            for layer in ls["layer_set"]:
                cfg[layer] = c
        return cfg

    @staticmethod
    def generate_block_pruner_config(d):
        return BlockPrunerConfig(d["sparsity"], d["block_height"], d["block_width"], d["sub_rows"],
                                 d["sub_cols"], d["collapse_tensor"])

    def generate_masks(self, model, is_static=False, verbose=False):
        sd = model.state_dict()
        for layer, pc in self.layer_configs.items():
            w = sd[layer].detach().cpu().numpy()
            if verbose:
                how = "static approach" if is_static else "pruning approach"
                print(f"Generating mask for layer {layer} using {how}")
            fn = BlockPruner.generate_mask_by_construction if is_static else BlockPruner.generate_mask_by_pruning
            self._store(layer, fn(w, pc))

    @staticmethod
    def generate_mask_by_pruning(tensor, pconfig, rev_mask=False):
        return BlockPruner._block_mask(tensor, pconfig, rev_mask, construct=False)

    @staticmethod
    def generate_mask_by_construction(tensor, pconfig, rev_mask=False):
        return BlockPruner._block_mask(tensor, pconfig, rev_mask, construct=True)

    @staticmethod
    def prune_tensor_as_block(tensor, sparsity, block_height, block_width, sub_rows=-1, sub_cols=-1,
                              collapse_tensor=True, rev_mask=False, dump_fpath=None):
        pc = BlockPrunerConfig(sparsity, block_height, block_width, sub_rows, sub_cols, collapse_tensor)
        return BlockPruner._block_mask(tensor, pc, rev_mask, construct=False, dump_fpath=dump_fpath)

    @staticmethod
    def construct_tensor_as_block(tensor, sparsity, block_height, block_width, sub_rows=-1, sub_cols=-1,
                                  collapse_tensor=True, rev_mask=False, dump_fpath=None):
        pc = BlockPrunerConfig(sparsity, block_height, block_width, sub_rows, sub_cols, collapse_tensor)
        return BlockPruner._block_mask(tensor, pc, rev_mask, construct=True, dump_fpath=dump_fpath)

    @staticmethod
    def _block_mask(tensor, pc, rev_mask, construct, dump_fpath=None):
        """BlockPruner.py:139-241 (prune) / :251-341 (construct)."""
        sp = pc.sparsity
        assert 0 <= sp <= 1, "Sparsity should be within [0,1]"
        tensor = np.asarray(tensor)
        mat = tensor.reshape(tensor.shape[0], tensor.size // tensor.shape[0])
        rows, cols = mat.shape
        unit = tensor.size // (tensor.shape[0] * tensor.shape[1])   # kh*kw for a conv weight
        bh = rows if pc.block_height == -1 else pc.block_height
        srows = rows if pc.sub_rows == -1 else pc.sub_rows
        bw = cols if pc.block_width == -1 else (pc.block_width if pc.collapse_tensor else pc.block_width * unit)
        scols = cols if pc.sub_cols == -1 else (pc.sub_cols if pc.collapse_tensor else pc.sub_cols * unit)

        if (rows, cols) == (srows, scols):
            mask = BlockPruner._base_mask(mat, sp, bh, bw, construct)
        else:
            if rows % srows or cols % scols:
                raise ValueError(f"sub-matrix {srows}x{scols} must tile the {rows}x{cols} matrix "
                                 "(the reference recursion does not terminate otherwise)")
            mask = np.zeros((rows, cols), dtype=mat.dtype)
            sub = BlockPrunerConfig(sp, bh, bw, srows, scols, True)
            for rb in range(rows // srows):          # row-major: same RNG order as the reference
                for cb in range(cols // scols):
                    rs, cs = slice(rb * srows, (rb + 1) * srows), slice(cb * scols, (cb + 1) * scols)
                    mask[rs, cs] = BlockPruner._block_mask(mat[rs, cs], sub, False, construct)
        if rev_mask:
            mask = (mask + 1) % 2
        if dump_fpath is not None:
            BlockPruner.write_block_matrix_to_file(BlockPruner.generate_block_matrix(mat * mask, bh, bw),
                                                   dump_fpath)
        return mask.reshape(tensor.shape)

    @staticmethod
    def _base_mask(mat, sp, bh, bw, construct):
        rows, cols = mat.shape
        if sp <= 0:
            return np.ones((rows, cols), dtype=mat.dtype)
        nrb, ncb = -(-rows // bh), -(-cols // bw)
        if construct:
            nnzb = int((1.0 - sp) * (nrb * ncb))
            keep = np.zeros(nrb * ncb, dtype=bool)
            keep[np.random.choice(nrb * ncb, nnzb, replace=False)] = True
            keep = keep.reshape(nrb, ncb)
        else:
            meta = mat if (bh, bw) == (1, 1) else _block_abs_sums(mat, bh, bw)
            absm = np.abs(meta)
            thresh = np.sort(absm.reshape(-1))[max(0, int(sp * meta.size) - 1)]
            keep = absm > thresh
        if (bh, bw) == (1, 1):
            return keep.astype(mat.dtype)
        return _expand_blocks(keep, bh, bw, rows, cols, mat.dtype)

    @staticmethod
    def generate_block_matrix(mat, block_height, block_width):
        """Dense -> BSR (BlockPruner.py:343-413): nonzero blocks row-major, values column-major
        within a block, block-column indices, rowBlockPtr."""
        assert mat.ndim == 2
        rows, cols = mat.shape
        if block_height == 1 and block_width == 1:
            r, c = np.nonzero(mat)
            values = mat[r, c].astype(mat.dtype)
            indices = c.astype(int)
            counts = np.bincount(r, minlength=rows + 1)[:rows + 1].astype(int)
        else:
            sums = _block_abs_sums(mat, block_height, block_width)
            nrb, ncb = sums.shape
            nz_r, nz_c = np.nonzero(sums)
            nnzb = nz_r.size
            values = np.zeros(nnzb * block_height * block_width, dtype=mat.dtype)
            for i, (rb, cb) in enumerate(zip(nz_r, nz_c)):
                blk = mat[rb * block_height:min(rows, (rb + 1) * block_height),
                          cb * block_width:min(cols, (cb + 1) * block_width)]
                flat = blk.flatten("F")
                base = i * block_height * block_width
                values[base:base + flat.size] = flat
            indices = nz_c.astype(int)
            counts = np.zeros(nrb + 1, dtype=int)
            counts[:nrb] = np.bincount(nz_r, minlength=nrb)
        ptr = np.zeros_like(counts)
        ptr[1:] = np.cumsum(counts[:-1])
        return BlockMatrix(rows, cols, block_height, block_width, values, indices, ptr)

    @staticmethod
    def write_block_matrix_to_file(block_mat, filepath="block_data.txt"):
        """Text BSR format (BlockPruner.py:415-432; fixture pruners/block_test.txt)."""
        nnzb = block_mat.rowBlockPtr[-1]
        with open(filepath, "w") as fh:
            for v in (block_mat.rows, block_mat.cols, block_mat.bh, block_mat.bw, nnzb):
                fh.write(str(v) + "\n")
            for arr in (block_mat.values, block_mat.indices, block_mat.rowBlockPtr):
                fh.write("".join(str(e) + " " for e in arr) + "\n")


# ============================================================================ RmbPruner
class BlockletType:
    def __init__(self, bh, bw):
        self.bh, self.bw = bh, bw

    def __str__(self):
        return "{}x{}".format(self.bh, self.bw)


class RmbPrunerConfig:
    def __init__(self, bh, bw, spo, bl_types, bl_counts):
        self.bh, self.bw, self.spo = bh, bw, spo
        self.bl_types, self.bl_counts = bl_types, bl_counts


class RmbPruner(Pruner):
    def parse_config_file(self, config_fp):
        cfg = collections.OrderedDict()
        for ls in _load_configs(config_fp)["configs"]:
            types = [BlockletType(b["bh"], b["bw"]) for b in ls["blocklets"]]
            counts = [b["count"] for b in ls["blocklets"]]
            c = RmbPrunerConfig(ls["global_bh"], ls["global_bw"], ls["global_sp"], types, counts)
            for layer in ls["layer_set"]:
                cfg[layer] = c
        return cfg

    def generate_masks(self, model, is_static=False, verbose=False):
        sd = model.state_dict()
        for layer, rc in self.layer_configs.items():
            if verbose:
                print("Generating mask for layer {}".format(layer))
            self._store(layer, RmbPruner.prune_tensor_as_rmb(sd[layer].detach().cpu().numpy(), rc))

    @staticmethod
    def prune_tensor_as_rmb(tensor, config, dump_fpath=None):
        """RmbPruner.py:127-243 for all blocks at once.

        Outer sparsity: per block-row, drop blocks whose |sum| <= the int(spo*ncb)-th
        smallest (:146-164).  Inner: for each blocklet type x count, in every
        blocklet-row of every kept block pick the column blocklet with the largest |sum|
        (first on ties), keep it, and zero it in the working copy (:189-226)."""
        tensor = np.asarray(tensor)
        mat = tensor.reshape(tensor.shape[0], -1).copy()
        rows, cols = mat.shape
        bh, bw = config.bh, config.bw
        assert rows % bh == 0, "Block height should divide rows"
        assert cols % bw == 0, "Block width should divide columns"
        nrb, ncb = rows // bh, cols // bw
        keep_blk = np.ones((nrb, ncb), dtype=bool)
        if config.spo > 0:
            meta = _block_abs_sums(mat, bh, bw).astype(np.float64) if (bh != 1 and bw != 1) \
                else np.abs(mat).astype(np.float64)
            ti = int(config.spo * meta.shape[1]) - 1
            if ti >= 0:
                th = np.sort(np.abs(meta), axis=1)[:, ti:ti + 1]
                keep_blk &= ~(meta <= th)
        mask = np.zeros(mat.shape, dtype=mat.dtype)
        # blocks as [nrb, ncb, bh, bw] views into the working copy
        work = mat.reshape(nrb, bh, ncb, bw).transpose(0, 2, 1, 3)
        mview = mask.reshape(nrb, bh, ncb, bw).transpose(0, 2, 1, 3)
        for t, cnt in zip(config.bl_types, config.bl_counts):
            lbh, lbw = t.bh, t.bw
            lnr, lnc = bh // lbh, bw // lbw
            for _ in range(cnt):
                for lr in range(lnr):
                    strip = work[:, :, lr * lbh:(lr + 1) * lbh, :lnc * lbw]
                    sub = np.abs(strip).reshape(nrb, ncb, lbh, lnc, lbw).transpose(0, 1, 3, 2, 4)
                    sums = np.ascontiguousarray(sub).reshape(nrb, ncb, lnc, lbh * lbw).sum(axis=3)
                    choice = np.argmax(sums.astype(np.float64), axis=2)       # [nrb, ncb]
                    rr, cc = np.nonzero(keep_blk)
                    ch = choice[rr, cc]
                    for dr in range(lbh):
                        for dc in range(lbw):
                            work[rr, cc, lr * lbh + dr, ch * lbw + dc] = 0
                            mview[rr, cc, lr * lbh + dr, ch * lbw + dc] = 1
        if dump_fpath is not None:
            RmbPruner._dump(tensor.reshape(tensor.shape[0], -1), config, keep_blk, dump_fpath)
        return mask.reshape(tensor.shape)

    @staticmethod
    def _dump(orig, config, keep_blk, path):
        """RMB text format (RmbPruner.py:246-378), rebuilt by replaying the selection."""
        mat = orig.copy()
        rows, cols = mat.shape
        bh, bw = config.bh, config.bw
        nrb, ncb = rows // bh, cols // bw
        blets = []   # (grb, gcb, lbh, lbw, values[bh, lbw], indices[lnr])
        for rb, cb in itertools.product(range(nrb), range(ncb)):
            if not keep_blk[rb, cb]:
                continue
            loc = mat[rb * bh:(rb + 1) * bh, cb * bw:(cb + 1) * bw]
            for t, cnt in zip(config.bl_types, config.bl_counts):
                lnr, lnc = bh // t.bh, bw // t.bw
                for _ in range(cnt):
                    vals = np.zeros((bh, t.bw))
                    idx = np.zeros(lnr)
                    for lr in range(lnr):
                        strip = loc[lr * t.bh:(lr + 1) * t.bh]
                        s = np.array([np.sum(np.abs(strip[:, j * t.bw:(j + 1) * t.bw])) for j in range(lnc)],
                                     dtype=np.float64)
                        ch = int(np.argmax(s))
                        vals[lr * t.bh:(lr + 1) * t.bh] = strip[:, ch * t.bw:(ch + 1) * t.bw]
                        idx[lr] = ch
                        strip[:, ch * t.bw:(ch + 1) * t.bw] = 0
                    blets.append((rb, cb, t.bh, t.bw, vals, idx))
        order = sorted(range(len(blets)), key=lambda i: blets[i][0] * ncb + blets[i][1])
        blets = [blets[i] for i in order]
        mbl_ids = [b[0] * ncb + b[1] for b in blets]
        uniq = sorted(set(mbl_ids))
        nnzb = len(uniq)
        per = collections.OrderedDict((u, [b for b, m in zip(blets, mbl_ids) if m == u]) for u in uniq)
        indices = np.array([u % ncb for u in uniq], dtype=int)
        rbp = np.zeros(nrb + 1, dtype=int)
        for u in uniq:
            rbp[u // ncb] += 1
        rbp[1:] = np.cumsum(rbp[:-1])
        rbp[0] = 0
        row_p = [int(round(np.log2(bh // b[2]))) for b in blets]
        col_p = [int(round(np.log2(bw // b[3]))) for b in blets]
        valc = [sum(b[4].size for b in per[u]) for u in uniq]
        indc = [sum(b[5].size for b in per[u]) for u in uniq]
        bltc = [len(per[u]) for u in uniq]

        def ptr(counts):
            p = np.zeros(nnzb + 1, dtype=int)
            p[:nnzb] = counts
            p[1:] = np.cumsum(p[:-1])
            p[0] = 0
            return p
        values = np.concatenate([b[4].flatten("F") for b in blets]) if blets else np.zeros(0)
        l_idx = np.concatenate([b[5].flatten("F") for b in blets]).astype(int) if blets else np.zeros(0, int)
        with open(path, "w") as fh:
            for v in (rows, cols, bh, bw, values.size, nnzb, len(blets), l_idx.size):
                fh.write(str(v) + "\n")
            for arr in (values, indices, rbp, row_p, col_p, l_idx, ptr(valc), ptr(indc), ptr(bltc)):
                fh.write("".join(str(e) + " " for e in arr) + "\n")


# ============================================================================ SRMBRepMasker
class SRMBRepMaskerConfig:
    def __init__(self, obh, obw, cbh, cbw, ibh, ibw, osp, opat, isp, ipat, is_repetitive, collapse_tensor,
                 cross_prob, is_symmetric):
        self.obh, self.obw, self.cbh, self.cbw, self.ibh, self.ibw = obh, obw, cbh, cbw, ibh, ibw
        self.osp, self.opat, self.isp, self.ipat = osp, opat, isp, ipat
        self.is_repetitive, self.collapse_tensor = is_repetitive, collapse_tensor
        self.cross_prob, self.is_symmetric = cross_prob, is_symmetric


class SRMBRepMasker(Pruner):
    _KEYS = ("obh", "obw", "cbh", "cbw", "ibh", "ibw", "osp", "opat", "isp", "ipat", "is_repetitive",
             "collapse_tensor", "cross_prob", "is_symmetric")

    def parse_config_file(self, config_fp):
        cfg = collections.OrderedDict()
        for ls in _load_configs(config_fp)["configs"]:
            c = SRMBRepMaskerConfig(*[ls[k] for k in self._KEYS])
            for layer in ls["layer_set"]:
                cfg[layer] = c
        return cfg

    def generate_masks(self, model, is_static=True, verbose=False):
        sd = model.state_dict()
        for layer, c in self.layer_configs.items():
            fac = SRMBRepMasker.mask_factors(sd[layer].detach().cpu().numpy(), c)
            self._store(layer, SRMBRepMasker.expand_factors(fac))
            self._factors[layer] = fac          # compact (period-tile) form for save_masks
            if verbose:
                print("Generated mask for layer {}".format(layer))

    @staticmethod
    def get_ramanujan_pattern(rows, cols, d, cross_prob=0.5, is_symmetric=False, debug=False):
        """Bi-regular lifted pattern (SRMBRepMasker.py:102-168): start from a dense
        (rows/(cols/d)) x d block, then repeatedly double it block-diagonally and, for each
        nonzero of the top-left quarter (row-major; upper triangle when symmetric), cross it
        with probability cross_prob (one binomial draw per nonzero, in scan order)."""
        assert cols % d == 0
        assert (cols // d) & (cols // d - 1) == 0
        assert rows // (cols // d) > 0
        if is_symmetric:
            assert rows == cols, "When symmetric, #rows = #cols"
        mask = np.zeros((rows, cols), dtype=int)
        cr, cc = rows // (cols // d), d
        mask[:cr, :cc] = 1
        while cc < cols:
            mask[cr:2 * cr, cc:2 * cc] = mask[:cr, :cc]
            quad = mask[:cr, :cc]
            if is_symmetric:
                sel = np.triu(np.ones((cr, cc), dtype=bool))
                ls, rs = np.nonzero((quad == 1) & sel)
            else:
                ls, rs = np.nonzero(quad == 1)
            draws = np.random.binomial(1, cross_prob, size=ls.size) if ls.size else np.zeros(0, int)
            for l, r, x in zip(ls, rs, draws):
                if x != 1:
                    continue
                mask[l, r] = 0
                mask[l + cr, r + cc] = 0
                mask[l, r + cc] = 1
                mask[l + cr, r] = 1
                if is_symmetric:
                    mask[r, l] = 0
                    mask[r + cc, l + cr] = 0
                    mask[r + cc, l] = 1
                    mask[r, l + cr] = 1
            cr, cc = 2 * cr, 2 * cc
        return mask

    @staticmethod
    def generate_sparsity_pattern(M, N, sparsity, pattern, cross_prob=0.5, is_symmetric=False):
        """SRMBRepMasker.py:171-334, same RNG calls in the same order."""
        nnz = M * int((1.0 - sparsity) * N)
        per_row = nnz // M
        mask = np.zeros((M, N))
        if sparsity == 0:
            mask[:] = 1
            return mask
        if pattern == "RANDOM":
            mask.reshape(M * N)[np.random.choice(M * N, nnz, replace=False)] = 1
        elif pattern == "UROW":
            assert nnz % M == 0
            for i in range(M):
                mask[i, np.random.choice(N, per_row, replace=False)] = 1
        elif pattern == "RAMANUJAN":
            mask = SRMBRepMasker.get_ramanujan_pattern(M, N, per_row, cross_prob, is_symmetric)
        elif pattern == "TRANS":
            assert nnz % M == 0
            assert M == N, "Matrix should be square"
            mask = SRMBRepMasker._trans(M, N, per_row)
        elif pattern == "CDIA":
            assert nnz % M == 0
            base = np.random.choice(N, per_row, replace=False)
            for i in range(M):
                mask[i, (i + base) % N] = 1
        elif pattern == "CDIASTRIDE":
            assert nnz % M == 0
            base = np.arange(0, N, N // per_row)
            for i in range(M):
                mask[i, (i + base) % N] = 1
        elif pattern == "COLUMN":
            assert nnz % M == 0
            mask[:, np.random.choice(N, per_row, replace=False)] = 1
        elif pattern == "CBAND":
            assert nnz % M == 0
            k = per_row // 2
            base = (np.arange(-k, k) + N) % N
            for i in range(M):
                mask[i, (i + base) % N] = 1
        elif pattern == "CCDIA":
            assert nnz % M == 0
            base = np.arange(per_row)
            for i in range(M):
                mask[i, (i + base) % N] = 1
        elif pattern == "CCOLUMN":
            assert nnz % M == 0
            mask[:, :per_row] = 1
        elif pattern == "GROUP":
            groups = N // per_row
            sh = M // groups
            for g in range(groups):
                mask[g * sh:(g + 1) * sh, g * per_row:(g + 1) * per_row] = 1
        else:
            raise ValueError("Unsupported {}".format(pattern))   # reference: print + exit(-1)
        return mask

    @staticmethod
    def _trans(M, N, per_row):
        """TRANS pattern (SRMBRepMasker.py:193-263)."""
        mask = np.zeros((M, N))
        if per_row <= int(0.25 * N):
            print("Truly random")
            xs = np.arange(M)
            for _ in range(per_row):
                while True:
                    ys = np.random.permutation(M)
                    if np.sum(mask[xs, ys]) == 0:
                        mask[xs, ys] = 1
                        break
            return mask
        mask += 1
        deg = np.ones(N, dtype=int) * M
        pool = np.arange(N)
        psize = N
        drop = N - per_row
        for u in range(M):
            chosen = np.zeros(N)
            for _ in range(drop):
                cand = pool[:psize]
                cdeg = deg[cand]
                locs = np.where(cdeg == np.max(cdeg))[0]
                while True:
                    ind = locs[np.random.randint(locs.size)]
                    v = cand[ind]
                    if chosen[v] == 0:
                        mask[u, v] = 0
                        chosen[v] = 1
                        deg[v] -= 1
                        if deg[v] == per_row:
                            last = pool[psize - 1]
                            pool[psize - 1] = pool[ind]
                            pool[ind] = last
                            psize -= 1
                        break
        return mask

    @staticmethod
    def construct_mask(tensor, config):
        """mask = kron(kron(OB, kron(CB, P)), IB) (SRMBRepMasker.py:337-383)."""
        return SRMBRepMasker.expand_factors(SRMBRepMasker.mask_factors(tensor, config))

    @staticmethod
    def mask_factors(tensor, config):
        """The mask's Kronecker factors, drawing the RNG exactly as SRMBRepMasker.py:337-383 does:
        repetitive masks are kron(kron(OB, kron(1(obh/cbh x obw/cbw), P)), 1(ibh x ibw*k)) -- an OB
        pattern over a period tile P, so OB and P (bits) and the block sizes ARE the mask; the
        non-repetitive form keeps its (rows/ibh x cols/ibw) block pattern OCP."""
        tensor = np.asarray(tensor)
        rows, cols = tensor.shape[0], tensor.shape[1]
        ks = tensor.size // (rows * cols)
        if config.collapse_tensor:
            cols *= ks
            ks = 1
        obh = rows if config.obh == -1 else config.obh
        obw = cols if config.obw == -1 else config.obw
        cbh = obh if config.cbh == -1 else config.cbh
        cbw = obw if config.cbw == -1 else config.cbw
        ibh, ibw = config.ibh, config.ibw
        gen = SRMBRepMasker.generate_sparsity_pattern
        ob = gen(rows // obh, cols // obw, config.osp, config.opat, config.cross_prob, config.is_symmetric)
        fac = {"shape": tuple(tensor.shape), "dtype": str(tensor.dtype), "ib": (ibh, ibw * ks),
               "rep": bool(config.is_repetitive)}
        if config.is_repetitive:
            p = gen(cbh // ibh, cbw // ibw, config.isp, config.ipat, config.cross_prob, config.is_symmetric)
            fac.update(ob=ob, cb=(obh // cbh, obw // cbw), p=p)
            return fac
        ocp = np.zeros((rows // ibh, cols // ibw), dtype=tensor.dtype)
        cb = np.ones((obh // cbh, obw // cbw), dtype=tensor.dtype)
        snr, snc = obh // ibh, obw // ibw
        for rb in range(rows // obh):
            for cb_ in range(cols // obw):
                if ob[rb, cb_] == 1:
                    p = gen(cbh // ibh, cbw // ibw, config.isp, config.ipat, config.cross_prob,
                            config.is_symmetric)
                    ocp[rb * snr:(rb + 1) * snr, cb_ * snc:(cb_ + 1) * snc] += np.kron(cb, p)
        fac.update(ocp=ocp)
        return fac

    @staticmethod
    def expand_factors(fac):
        """The full weight-shaped mask from mask_factors() (the reference's kron, same dtypes)."""
        dt = np.dtype(fac["dtype"])
        ib = np.ones(fac["ib"], dtype=dt)
        if fac["rep"]:
            cb = np.ones(fac["cb"], dtype=dt)
            m = np.kron(np.kron(fac["ob"], np.kron(cb, fac["p"])), ib)
            return m.reshape(fac["shape"]).astype(dt)
        return np.kron(fac["ocp"].astype(dt), ib).reshape(fac["shape"])


__all__ = ["Pruner", "BlockPruner", "BlockPrunerConfig", "BlockMatrix", "RmbPruner", "RmbPrunerConfig",
           "BlockletType", "SRMBRepMasker", "SRMBRepMaskerConfig", "make_pruner"]
