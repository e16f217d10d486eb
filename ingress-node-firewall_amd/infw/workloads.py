"""Synthetic workloads of BASELINE.json configs, backed by
libinfw_workload.so: table entries (keys + interned rule templates), frame
header snapshots for the oracle, host tuples, and an on-device SoA generator.
Packet i is a pure function of (seed, i), so shards are reproducible at any
GPU count.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _native as N

CFG0_DEMO, CFG1_V4_10K, CFG2_MIXED_1M, CFG4_ADVERSARIAL = 0, 1, 2, 4
SEEDS = {CFG0_DEMO: 0x1F000000, CFG1_V4_10K: 0x1F000001, CFG2_MIXED_1M: 0x1F000002, CFG4_ADVERSARIAL: 0x1F000004}


def _threads() -> int:
    return max(1, min(16, os.cpu_count() or 1))


class Workload:
    def __init__(self, cfg: int, seed: int | None = None, n_prefixes: int = 0, n_templates: int = 0):
        self.cfg = cfg
        self.seed = SEEDS[cfg] if seed is None else seed
        self._h = C.c_void_p()
        N.check(N.wl.infw_wl_create(C.byref(self._h), cfg, self.seed, n_prefixes, n_templates), "infw_wl_create")
        self._uploaded = None

    def close(self):
        if self._h:
            N.wl.infw_wl_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- tables
    @property
    def n_entries(self) -> int:
        return int(N.wl.infw_wl_n_entries(self._h))

    @property
    def n_templates(self) -> int:
        return int(N.wl.infw_wl_n_templates(self._h))

    def keys_bytes(self) -> np.ndarray:
        return np.ctypeslib.as_array((C.c_uint8 * (24 * self.n_entries)).from_address(
            N.wl.infw_wl_keys(self._h))).copy()

    def val_index(self) -> np.ndarray:
        return np.ctypeslib.as_array((C.c_uint32 * self.n_entries).from_address(
            N.wl.infw_wl_val_index(self._h))).copy()

    def templates_bytes(self) -> np.ndarray:
        return np.ctypeslib.as_array((C.c_uint8 * (1200 * self.n_templates)).from_address(
            N.wl.infw_wl_templates(self._h))).copy()

    def load_into(self, classifier, flags: int = N.BPF_ANY, order=None) -> int:
        """Push every entry through the table-map update path (batched), in the workload's order or in `order`
        (a permutation of the entry indices).  The generator lists prefixes in popularity order; the reference's
        loader updates keys in Go map order (loader.go:158-208: a map range, i.e. random), which a shuffled
        order reproduces — list ids are assigned in first-update order, so the order places the decision lines."""
        if order is None:
            return classifier.update_batch_ptr(N.wl.infw_wl_keys(self._h), N.wl.infw_wl_templates(self._h),
                                               N.wl.infw_wl_val_index(self._h), self.n_entries, flags)
        order = np.asarray(order, dtype=np.int64)
        keys = np.ascontiguousarray(self.keys_bytes().reshape(-1, 24)[order])
        vi = np.ascontiguousarray(self.val_index()[order])
        return classifier.update_batch_ptr(keys.ctypes.data, N.wl.infw_wl_templates(self._h), vi.ctypes.data,
                                           len(order), flags)

    def shuffled_order(self, seed: int = 0x5EED) -> np.ndarray:
        """The entries that survive a load in workload order — for every LPM entry (prefixLen, ifindex and the
        first prefixLen - 32 address bits; host bits ignored) its last update, which also fixes the host bits the
        map keeps — in a seeded random order.  Loading these gives the same map as load_into() without `order`."""
        kb = self.keys_bytes().reshape(-1, 24)
        plen = kb[:, 0:4].copy().view("<u4").ravel().astype(np.int64)
        bits = np.clip(plen[:, None] - 32 - 8 * np.arange(16)[None, :], 0, 8)          # address bits kept per byte
        mask = ((0xFF00 >> bits) & 0xFF).astype(np.uint8)
        masked = np.concatenate([kb[:, :8], kb[:, 8:] & mask], axis=1)
        rows = np.ascontiguousarray(masked).view(np.dtype((np.void, 24))).ravel()
        _, last_rev = np.unique(rows[::-1], return_index=True)
        last = (len(rows) - 1 - last_rev).astype(np.int64)
        return np.random.default_rng(seed).permutation(last)

    def entries(self):
        """(key bytes[24], value bytes[1200]) pairs in update order."""
        kb, vi, tb = self.keys_bytes().reshape(-1, 24), self.val_index(), self.templates_bytes().reshape(-1, 1200)
        for i in range(kb.shape[0]):
            yield kb[i].tobytes(), tb[vi[i]].tobytes()

    def params(self) -> N.GenParams:
        return N.wl.infw_wl_params(self._h).contents

    def uniform_sources(self) -> None:
        """Draw sources uniformly over the prefixes (no Zipf head); tables unchanged."""
        N.wl.infw_wl_uniform_sources(self._h)

    def set_packet_seed(self, seed: int) -> None:
        N.wl.infw_wl_set_packet_seed(self._h, seed)

    # --- packets
    def frames(self, start: int, n: int):
        """Header snapshots (n x 80 B), linear length, frame length, ifindex."""
        hdr = np.zeros((n, N.HDR_SNAP), np.uint8)
        cap, plen, ifx = (np.zeros(n, np.uint32) for _ in range(3))
        N.check(N.wl.infw_wl_frames(self._h, start, n, hdr.ctypes.data, cap.ctypes.data, plen.ctypes.data,
                                    ifx.ctypes.data, _threads()), "frames")
        return hdr, cap, plen, ifx

    def gen_frames_device(self, frames, stride: int, linear_len, pkt_len, ifindex, start: int, dev_ordinal: int,
                          stream=None) -> None:
        """Raw frames of packets [start, start + n) in device memory at a fixed stride (n = linear_len.numel()):
        frame i = the 80-B header snapshot of frames(); linear_len = min(linear length, 80)."""
        if self._uploaded != dev_ordinal:
            N.check(N.wl.infw_wl_upload(self._h, dev_ordinal), "wl upload")
            self._uploaded = dev_ordinal
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(frames.device)
        sp = stream if isinstance(stream, int) else stream.cuda_stream
        N.check(N.wl.infw_wl_gen_frames(self._h, start, linear_len.numel(), frames.data_ptr(), stride,
                                        linear_len.data_ptr(), pkt_len.data_ptr(), ifindex.data_ptr(), sp),
                "gen_frames")

    def tuples(self, start: int, n: int) -> np.ndarray:
        t = np.zeros((n, 8), np.uint32)
        N.check(N.wl.infw_wl_tuples(self._h, start, n, t.ctypes.data, _threads()), "tuples")
        return t

    def gen_device(self, batch, start: int, dev_ordinal: int, stream=None) -> None:
        """Fill a SoaBatch with packets [start, start + batch.n) on the device."""
        if self._uploaded != dev_ordinal:
            N.check(N.wl.infw_wl_upload(self._h, dev_ordinal), "wl upload")
            self._uploaded = dev_ordinal
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(batch.device)
        sp = stream if isinstance(stream, int) else stream.cuda_stream
        N.check(N.wl.infw_wl_gen_soa(self._h, start, batch.n, batch.saddr.data_ptr(), batch.ifindex.data_ptr(),
                                     batch.pkt_len.data_ptr(), batch.meta.data_ptr(), batch.l4word.data_ptr(),
                                     sp), "gen_soa")


def pack_frames(hdr: np.ndarray, caplen: np.ndarray, pkt_len: np.ndarray, ifindex: np.ndarray) -> np.ndarray:
    """Frame header snapshots -> tuples (the product's raw-frame packer, host side)."""
    n = hdr.shape[0]
    h = np.zeros((n, N.HDR_SNAP), np.uint8)
    w = min(hdr.shape[1], N.HDR_SNAP)
    h[:, :w] = hdr[:, :w]
    t = np.zeros((n, 8), np.uint32)
    cap = np.ascontiguousarray(caplen, np.uint32)
    pl = np.ascontiguousarray(pkt_len, np.uint32)
    ifx = np.ascontiguousarray(ifindex, np.uint32)
    N.check(N.wl.infw_wl_pack(h.ctypes.data, cap.ctypes.data, pl.ctypes.data, ifx.ctypes.data, n, t.ctypes.data),
            "pack")
    return t


def line_rates(dev_ordinal: int) -> dict:
    """The device's random-line and stream rates measured now, in this process (infw_wl_line_rates, ~0.3 s):
    independent random 16-B lookups hitting the L2 (1-MiB table) and missing it (2-GiB table), and coalesced
    non-temporal stream reads — what bench.py's random_line_model prices the kernel's PMC line counts with."""
    out = (C.c_double * 3)()
    N.check(N.wl.infw_wl_line_rates(dev_ordinal, out), "line_rates")
    return {"l2_hit_G_per_s": round(out[0], 1), "l2_miss_G_per_s": round(out[1], 1), "stream_GB_per_s": round(out[2], 1)}
