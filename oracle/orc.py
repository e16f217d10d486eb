"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/build/liborc.so (oracle/infw_oracle.c), the CPU
restatement of bpf/ingress_node_firewall_kernel.c and of the LPM-trie map it
runs against.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg import this module, and only as the checker.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "liborc.so")
if not os.path.exists(LIB_PATH):
    raise ImportError(f"{LIB_PATH} not built: run `make`")
_lib = C.CDLL(LIB_PATH)

P = C.POINTER
_sig = {
    "orc_map_create": (C.c_void_p, [C.c_uint32]),
    "orc_map_destroy": (None, [C.c_void_p]),
    "orc_map_update": (C.c_int, [C.c_void_p, C.c_char_p, C.c_char_p, C.c_uint64]),
    "orc_map_delete": (C.c_int, [C.c_void_p, C.c_char_p]),
    "orc_map_lookup": (C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p]),
    "orc_map_get_next_key": (C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p]),
    "orc_map_count": (C.c_uint64, [C.c_void_p]),
    "orc_xdp_run": (C.c_int, [C.c_void_p, C.c_void_p, C.c_char_p, C.c_uint32, C.c_uint32, C.c_uint32,
                              P(C.c_uint32), P(C.c_int)]),
    "orc_classify_frames": (C.c_double, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]),
    "orc_rules_examined": (C.c_uint64, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.c_void_p, C.c_uint64]),
    "orc_collect_events": (C.c_uint64, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64]),
    "orc_perf_sample": (C.c_uint32, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]),
    "orc_collect_lookup_keys": (C.c_uint64, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                             C.c_uint64, C.c_void_p, C.c_uint64]),
}
for _n, (_r, _a) in _sig.items():
    getattr(_lib, _n).restype = _r
    getattr(_lib, _n).argtypes = _a

class OrcEvent(C.Structure):
    _fields_ = [("pkt_index", C.c_uint64), ("ifId", C.c_uint16), ("ruleId", C.c_uint16), ("action", C.c_uint8),
                ("pad", C.c_uint8), ("pktLength", C.c_uint16), ("captured", C.c_uint16)]


STATS_DTYPE = np.uint64  # [1024, 4]: allow.packets, allow.bytes, deny.packets, deny.bytes


class OracleMap:
    """The table map + data path of the reference, on the CPU."""

    def __init__(self, max_entries: int = 1 << 22):
        self._m = _lib.orc_map_create(max_entries)

    def close(self):
        if self._m:
            _lib.orc_map_destroy(self._m)
            self._m = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def update(self, key: bytes, val: bytes, flags: int = 0) -> int:
        assert len(key) == 24 and len(val) == 1200
        return _lib.orc_map_update(self._m, bytes(key), bytes(val), flags)

    def delete(self, key: bytes) -> int:
        return _lib.orc_map_delete(self._m, bytes(key))

    def lookup(self, key: bytes):
        out = C.create_string_buffer(1200)
        rc = _lib.orc_map_lookup(self._m, bytes(key), out)
        return None if rc else out.raw

    def next_key(self, key):
        out = C.create_string_buffer(24)
        rc = _lib.orc_map_get_next_key(self._m, None if key is None else bytes(key), out)
        return None if rc else out.raw

    def keys(self):
        k = self.next_key(None)
        while k is not None:
            yield k
            k = self.next_key(k)

    def __len__(self):
        return int(_lib.orc_map_count(self._m))

    def run(self, frame: bytes, ifindex: int, buff_len: int | None = None, stats: np.ndarray | None = None):
        """One XDP invocation; returns (xdp_action, result_word, event_emitted)."""
        res = C.c_uint32(0)
        ev = C.c_int(0)
        sp = None if stats is None else stats.ctypes.data
        act = _lib.orc_xdp_run(self._m, sp, bytes(frame), len(frame), len(frame) if buff_len is None else buff_len,
                               ifindex, C.byref(res), C.byref(ev))
        return act, res.value, bool(ev.value)

    def classify_frames(self, hdr: np.ndarray, caplen: np.ndarray, pkt_len: np.ndarray, ifindex: np.ndarray,
                        nthreads: int = 1, want_results: bool = True):
        """Batch over header snapshots (n x W bytes).  Returns (results, verdicts, stats[1024,4], seconds)."""
        n = hdr.shape[0]
        h = np.ascontiguousarray(hdr, dtype=np.uint8)
        w = h.shape[1] if n else 0
        offs = (np.arange(n, dtype=np.uint64) * np.uint64(w))
        cap = np.minimum(np.ascontiguousarray(caplen, np.uint32), np.uint32(max(w, 0)))
        # the program never reads past byte 74, so a snapshot of w >= 80 bytes stands in for the frame
        cap_full = np.ascontiguousarray(caplen, np.uint32) if w >= 80 else cap
        pl = np.ascontiguousarray(pkt_len, np.uint32)
        ifx = np.ascontiguousarray(ifindex, np.uint32)
        res = np.zeros(n, np.uint32) if want_results else None
        ver = np.zeros(n, np.uint8) if want_results else None
        stats = np.zeros((1024, 4), np.uint64)
        secs = _lib.orc_classify_frames(self._m, h.ctypes.data, offs.ctypes.data, cap_full.ctypes.data,
                                        pl.ctypes.data, ifx.ctypes.data, n,
                                        None if res is None else res.ctypes.data,
                                        None if ver is None else ver.ctypes.data, stats.ctypes.data, nthreads)
        return res, ver, stats, secs

    def rules_examined(self, hdr: np.ndarray, caplen: np.ndarray, pkt_len: np.ndarray, ifindex: np.ndarray) -> int:
        """Valid rules the reference's first-match loop looks at over the batch, up to and including each
        packet's first match (rule bytes examined = 12 B each)."""
        n = hdr.shape[0]
        h = np.ascontiguousarray(hdr, dtype=np.uint8)
        w = h.shape[1] if n else 0
        offs = np.arange(n, dtype=np.uint64) * np.uint64(w)
        cap = np.ascontiguousarray(caplen, np.uint32)
        cap = cap if w >= 80 else np.minimum(cap, np.uint32(max(w, 0)))
        pl = np.ascontiguousarray(pkt_len, np.uint32)
        ifx = np.ascontiguousarray(ifindex, np.uint32)
        return int(_lib.orc_rules_examined(self._m, h.ctypes.data, offs.ctypes.data, cap.ctypes.data,
                                           pl.ctypes.data, ifx.ctypes.data, n))

    def collect_events(self, hdr: np.ndarray, caplen: np.ndarray, pkt_len: np.ndarray, ifindex: np.ndarray,
                       max_events: int | None = None):
        """DENY events (kernel.c:392-399) in packet order: array of (pkt_index, ifId, ruleId, action, pktLength,
        captured)."""
        n = hdr.shape[0]
        h = np.ascontiguousarray(hdr, dtype=np.uint8)
        w = h.shape[1] if n else 0
        offs = np.arange(n, dtype=np.uint64) * np.uint64(w)
        cap = np.ascontiguousarray(caplen, np.uint32)
        pl = np.ascontiguousarray(pkt_len, np.uint32)
        ifx = np.ascontiguousarray(ifindex, np.uint32)
        m = n if max_events is None else max_events
        ev = (OrcEvent * max(m, 1))()
        k = _lib.orc_collect_events(self._m, h.ctypes.data, offs.ctypes.data, cap.ctypes.data, pl.ctypes.data,
                                    ifx.ctypes.data, n, ev, m)
        return np.array([(e.pkt_index, e.ifId, e.ruleId, e.action, e.pktLength, e.captured) for e in ev[:k]],
                        dtype=np.uint64).reshape(-1, 6)

    def collect_event_samples(self, buf: np.ndarray, offsets: np.ndarray, linear: np.ndarray, pkt_len: np.ndarray,
                              ifindex: np.ndarray):
        """DENY events of frames packed back to back in `buf` (frame i at offsets[i], linear[i] bytes) in packet
        order, and each event's perf sample (kernel.c:392-399): (events as in collect_events, k x 272 uint8)."""
        n = len(offsets)
        b = np.ascontiguousarray(buf, dtype=np.uint8)
        offs = np.ascontiguousarray(offsets, np.uint64)
        cap = np.ascontiguousarray(linear, np.uint32)
        pl = np.ascontiguousarray(pkt_len, np.uint32)
        ifx = np.ascontiguousarray(ifindex, np.uint32)
        ev = (OrcEvent * max(n, 1))()
        k = _lib.orc_collect_events(self._m, b.ctypes.data, offs.ctypes.data, cap.ctypes.data, pl.ctypes.data,
                                    ifx.ctypes.data, n, ev, n)
        out = np.zeros((k, 272), np.uint8)
        for j in range(k):
            i = ev[j].pkt_index
            _lib.orc_perf_sample(b.ctypes.data + int(offs[i]), int(min(cap[i], pl[i])), C.byref(ev[j]),
                                 out[j].ctypes.data)
        recs = np.array([(e.pkt_index, e.ifId, e.ruleId, e.action, e.pktLength, e.captured) for e in ev[:k]],
                        dtype=np.uint64).reshape(-1, 6)
        return recs, out


DBG_MAX_ENTRIES = 16384  # ingress_node_firewall_dbg_map max_entries (kernel.c:63)


def debug_map_after(hdr: np.ndarray, caplen: np.ndarray, pkt_len: np.ndarray, ifindex: np.ndarray,
                    max_entries: int = DBG_MAX_ENTRIES):
    """Contents of the dbg map after the frames ran in packet order on one CPU: BPF_NOEXIST
    inserts (kernel.c:214-216, :297-299) into a HASH of max_entries — the first max_entries
    distinct lookup keys, in first-seen order.  Also returns the number of distinct keys."""
    n = hdr.shape[0]
    h = np.ascontiguousarray(hdr, dtype=np.uint8)
    w = h.shape[1] if n else 0
    offs = np.arange(n, dtype=np.uint64) * np.uint64(w)
    cap = np.ascontiguousarray(caplen, np.uint32)
    pl = np.ascontiguousarray(pkt_len, np.uint32)
    ifx = np.ascontiguousarray(ifindex, np.uint32)
    out = np.zeros((max(n, 1), 24), np.uint8)
    k = _lib.orc_collect_lookup_keys(h.ctypes.data, offs.ctypes.data, cap.ctypes.data, pl.ctypes.data,
                                     ifx.ctypes.data, n, out.ctypes.data, n)
    seen = {}
    for row in out[:k]:
        b = row.tobytes()
        if b not in seen:
            seen[b] = None
    keys = list(seen)
    return keys[:max_entries], len(keys)
