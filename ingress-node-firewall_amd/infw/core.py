"""Classifier context: the table map, the batched data path and the statistics map.

Thin wrapper over libinfw's C ABI (include/infw.h).  Method names follow the
cilium/ebpf *Map calls the reference's pkg/ebpf makes on
ingress_node_firewall_table_map / ingress_node_firewall_statistics_map.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

import numpy as np

from . import _native as N
from ._native import LpmIpKeySt, RulesValSt, RuleStatisticsSt, check


def build_ebpf_key(if_id: int, cidr: str) -> LpmIpKeySt:
    """BuildEBPFKey (pkg/ebpf/ingress_node_firewall_loader.go:530-547)."""
    k = LpmIpKeySt()
    check(N.lib.infw_build_ebpf_key(C.c_uint32(if_id), cidr.encode(), C.byref(k)), f"BuildEBPFKey({cidr!r})")
    return k


def key_from_fields(prefix_len: int, ifindex: int, ip: bytes) -> LpmIpKeySt:
    k = LpmIpKeySt()
    k.prefixLen = prefix_len
    k.ingress_ifindex = ifindex
    b = bytes(ip)[:16]
    C.memmove(k.ip_data, b, len(b))
    return k


# Options applied to every Classifier created afterwards, before the caller's own `options` (include/infw.h
# infw_set_option).  A process that wants one form everywhere (a tool, a test) sets them once; the library itself
# reads no environment.
DEFAULT_OPTIONS: Dict[str, int] = {}


class Classifier:
    """One context = replicated GPU tables + one statistics slot per device.

    flags=F_HOST_ONLY gives a control-plane-only context (map API, compile,
    debug_walk) that works without a GPU; classify() then raises ENODEV.
    """

    def __init__(self, devices: Optional[Sequence[int]] = None, max_entries: int = 0, flags: int = 0,
                 options: Optional[Dict[str, int]] = None):
        self._ctx = C.c_void_p()
        arr = (C.c_int * len(devices))(*devices) if devices else None
        check(N.lib.infw_create(C.byref(self._ctx), arr, len(devices) if devices else 0, max_entries, flags),
              "infw_create")
        self._devices = list(devices) if devices else None
        for k, v in {**DEFAULT_OPTIONS, **(options or {})}.items():
            self.set_option(k, v)

    # -- per-context options (include/infw.h infw_set_option): bit-exact table forms and launch choices
    def set_option(self, name: str, value: int) -> None:
        check(N.lib.infw_set_option(self._ctx, name.encode(), int(value)), f"set_option({name}={value})")

    def option(self, name: str) -> int:
        v = C.c_int64(0)
        check(N.lib.infw_get_option(self._ctx, name.encode(), C.byref(v)), f"get_option({name})")
        return v.value

    def variant(self, input: int = N.INPUT_SOA, events: bool = False, dev: int = 0) -> str:
        """Registry name of the kernel instantiation(s) a launch would run (infw_classify_variant)."""
        buf = C.create_string_buffer(256)
        check(N.lib.infw_classify_variant(self._ctx, dev, input, N.VARIANT_EVENTS if events else 0, buf, 256),
              "classify_variant")
        return buf.value.decode()

    def launch_counts(self, dev: int = 0) -> tuple:
        """(two-phase launches, two-phase launches run as the fused kernel for want of scratch) since creation
        (infw_launch_counts)."""
        c = (C.c_uint64 * 2)()
        check(N.lib.infw_launch_counts(self._ctx, dev, c), "launch_counts")
        return int(c[0]), int(c[1])

    # -- lifecycle
    def close(self):
        if self._ctx:
            N.lib.infw_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def num_devices(self) -> int:
        return N.lib.infw_num_devices(self._ctx)

    # -- table map (cilium Map.Update / Delete / Lookup / Iterate)
    def update(self, key: LpmIpKeySt, val: RulesValSt, flags: int = N.BPF_ANY) -> None:
        check(N.lib.infw_table_update(self._ctx, C.byref(key), C.byref(val), flags), "Map.Update")

    def update_rc(self, key: LpmIpKeySt, val: RulesValSt, flags: int = N.BPF_ANY) -> int:
        return N.lib.infw_table_update(self._ctx, C.byref(key), C.byref(val), flags)

    def update_batch(self, keys, vals, val_index=None, flags: int = N.BPF_ANY) -> int:
        """keys: bytes/array of n*24 B; vals: bytes/array of m*1200 B; val_index: u32[n] or None."""
        kb = np.frombuffer(bytes(keys) if not isinstance(keys, np.ndarray) else keys.tobytes(), np.uint8)
        vb = np.frombuffer(bytes(vals) if not isinstance(vals, np.ndarray) else vals.tobytes(), np.uint8)
        n = kb.size // 24
        vi = None if val_index is None else np.ascontiguousarray(val_index, dtype=np.uint32)
        done = C.c_uint64(0)
        rc = N.lib.infw_table_update_batch(self._ctx, kb.ctypes.data, vb.ctypes.data,
                                           None if vi is None else vi.ctypes.data, n, flags, C.byref(done))
        check(rc, f"Map.BatchUpdate (applied {done.value} of {n})")
        return done.value

    def update_batch_ptr(self, keys_ptr: int, vals_ptr: int, val_index_ptr: Optional[int], n: int,
                         flags: int = N.BPF_ANY) -> int:
        done = C.c_uint64(0)
        check(N.lib.infw_table_update_batch(self._ctx, keys_ptr, vals_ptr, val_index_ptr, n, flags,
                                            C.byref(done)), "Map.BatchUpdate")
        return done.value

    def delete(self, key: LpmIpKeySt) -> None:
        check(N.lib.infw_table_delete(self._ctx, C.byref(key)), "Map.Delete")

    def delete_batch_ptr(self, keys_ptr: int, n: int) -> int:
        """infw_table_delete_batch over n packed 24-B keys at keys_ptr; returns the keys deleted (raises on the
        first error, like BPF_MAP_DELETE_BATCH)."""
        done = C.c_uint64(0)
        check(N.lib.infw_table_delete_batch(self._ctx, keys_ptr, n, C.byref(done)),
              f"Map.BatchDelete (deleted {done.value} of {n})")
        return done.value

    def delete_rc(self, key: LpmIpKeySt) -> int:
        return N.lib.infw_table_delete(self._ctx, C.byref(key))

    def lookup(self, key: LpmIpKeySt) -> Optional[RulesValSt]:
        v = RulesValSt()
        rc = N.lib.infw_table_lookup(self._ctx, C.byref(key), C.byref(v))
        if rc == -2:  # ENOENT
            return None
        check(rc, "Map.Lookup")
        return v

    def next_key(self, key: Optional[LpmIpKeySt]) -> Optional[LpmIpKeySt]:
        nk = LpmIpKeySt()
        rc = N.lib.infw_table_get_next_key(self._ctx, C.byref(key) if key is not None else None, C.byref(nk))
        if rc == -2:
            return None
        check(rc, "Map.NextKey")
        return nk

    def iterate(self) -> Iterator[Tuple[LpmIpKeySt, RulesValSt]]:
        """Map.Iterate(): get_next_key walk + lookup of each key (loader.go:293-296)."""
        k = self.next_key(None)
        while k is not None:
            v = self.lookup(k)
            if v is not None:
                yield k, v
            k = self.next_key(k)

    def count(self) -> int:
        n = C.c_uint64(0)
        check(N.lib.infw_table_count(self._ctx, C.byref(n)), "count")
        return n.value

    def commit(self) -> None:
        check(N.lib.infw_table_commit(self._ctx), "commit")

    def export_size(self) -> int:
        """Bytes of the committed epoch's image (infw_table_export with no buffer)."""
        n = C.c_uint64(0)
        check(N.lib.infw_table_export(self._ctx, None, 0, C.byref(n)), "table_export")
        return n.value

    def export_into(self, ptr: int, cap: int) -> int:
        """infw_table_export into caller memory at `ptr` (e.g. a shared mmap); returns the image size."""
        n = C.c_uint64(0)
        check(N.lib.infw_table_export(self._ctx, ptr, cap, C.byref(n)), "table_export")
        return n.value

    def export_image(self) -> bytes:
        """The committed epoch as an image another context (another rank's) can import."""
        buf = C.create_string_buffer(self.export_size())
        n = self.export_into(C.addressof(buf), len(buf))
        return buf.raw[:n]

    def import_image(self, image) -> None:
        """infw_table_import: install an exported epoch (bytes, or (ptr, size) of caller memory) on an empty
        context — its entries become the committed set and every device slot gets the tables, no compile."""
        if isinstance(image, tuple):
            ptr, size = image
            check(N.lib.infw_table_import(self._ctx, ptr, size), "table_import")
        else:
            b = bytes(image)
            check(N.lib.infw_table_import(self._ctx, b, len(b)), "table_import")

    def info(self) -> Dict[str, float]:
        ti = N.TableInfo()
        check(N.lib.infw_table_info(self._ctx, C.byref(ti)), "info")
        d = {f: getattr(ti, f) for f, _ in N.TableInfo._fields_ if f not in ("reserved0", "reserved1", "reserved")}
        d["full_reason"] = ti.full_reason.decode()
        return d

    # -- data path
    def classify_ptrs(self, dev: int, saddr: int, ifindex: int, pkt_len: int, meta: int, l4word: int, n: int,
                      results: int = 0, verdicts: int = 0, stream: int = 0) -> None:
        b = N.BatchSoa(saddr, ifindex, pkt_len, meta, l4word)
        check(N.lib.infw_classify(self._ctx, dev, C.byref(b), n, results or None, verdicts or None,
                                  stream or None), "classify")

    def classify(self, batch, results=None, verdicts=None, dev: int = 0, stream=None) -> None:
        """batch: infw.batch.SoaBatch (torch tensors on the device); results/verdicts: torch tensors or None.
        stream: torch.cuda.Stream or raw hipStream_t int; default torch's current stream."""
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(batch.device)
        sp = stream if isinstance(stream, int) else stream.cuda_stream
        self.classify_ptrs(dev, batch.saddr.data_ptr(), batch.ifindex.data_ptr(), batch.pkt_len.data_ptr(),
                           batch.meta.data_ptr(), batch.l4word.data_ptr(), batch.n,
                           results.data_ptr() if results is not None else 0,
                           verdicts.data_ptr() if verdicts is not None else 0, sp)

    def compact(self, batch, dev: int = 0, stream=None):
        """infw_soa_compact: a SoaBatchC of `batch` (address bytes re-laid out on the device, other streams shared)."""
        from .batch import SoaBatchC
        out = SoaBatchC.empty_for(batch)
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(batch.device)
        sp = stream if isinstance(stream, int) else stream.cuda_stream
        b = N.BatchSoa(batch.saddr.data_ptr(), batch.ifindex.data_ptr(), batch.pkt_len.data_ptr(),
                       batch.meta.data_ptr(), batch.l4word.data_ptr())
        check(N.lib.infw_soa_compact(self._ctx, dev, C.byref(b), batch.n, out.saddr4.data_ptr(), out.v6tail.data_ptr(),
                                     sp), "soa_compact")
        return out

    def classify_c(self, batch_c, results=None, verdicts=None, dev: int = 0, stream=None) -> None:
        """infw_classify_c over a SoaBatchC (identical results to classify on the standard layout)."""
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(batch_c.device)
        sp = stream if isinstance(stream, int) else stream.cuda_stream
        b = N.BatchSoaC(batch_c.saddr4.data_ptr(), batch_c.v6tail.data_ptr(), batch_c.ifindex.data_ptr(),
                        batch_c.pkt_len.data_ptr(), batch_c.meta.data_ptr(), batch_c.l4word.data_ptr())
        check(N.lib.infw_classify_c(self._ctx, dev, C.byref(b), batch_c.n,
                                    results.data_ptr() if results is not None else None,
                                    verdicts.data_ptr() if verdicts is not None else None, sp), "classify_c")

    def classify_events(self, batch, events, events_count, results=None, verdicts=None, dev: int = 0,
                        stream=None) -> None:
        """classify + the deny-event stream (kernel.c:392-399) into `events` (uint8 tensor of cap*24 B)
        and `events_count` (int64 tensor [1], incremented by the kernel)."""
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(batch.device)
        sp = stream if isinstance(stream, int) else stream.cuda_stream
        b = N.BatchSoa(batch.saddr.data_ptr(), batch.ifindex.data_ptr(), batch.pkt_len.data_ptr(),
                       batch.meta.data_ptr(), batch.l4word.data_ptr())
        ex = N.ClassifyEx(C.sizeof(N.ClassifyEx), 0, events.data_ptr(), events.numel() // C.sizeof(N.EventRec),
                          events_count.data_ptr())
        check(N.lib.infw_classify_ex(self._ctx, dev, C.byref(b), batch.n,
                                     results.data_ptr() if results is not None else None,
                                     verdicts.data_ptr() if verdicts is not None else None, C.byref(ex), sp),
              "classify_ex")

    def classify_host(self, soa: "HostSoa", results=None, verdicts=None, dev: int = 0, chunk: int = 0) -> None:
        """Host-resident batch (numpy arrays, see HostSoa): pipelined through the device in chunks; returns when
        results (uint32 array) / verdicts (uint8 array) are filled."""
        b = N.BatchSoa(soa.saddr.ctypes.data, soa.ifindex.ctypes.data, soa.pkt_len.ctypes.data,
                       soa.meta.ctypes.data, soa.l4word.ctypes.data)
        check(N.lib.infw_classify_host(self._ctx, dev, C.byref(b), soa.n,
                                       results.ctypes.data if results is not None else None,
                                       verdicts.ctypes.data if verdicts is not None else None, chunk),
              "classify_host")

    def host_register(self, arr: np.ndarray) -> None:
        """Page-lock a numpy array's memory for full-rate infw_classify_host copies."""
        check(N.lib.infw_host_register(self._ctx, arr.ctypes.data, arr.nbytes), "host_register")

    def host_unregister(self, arr: np.ndarray) -> None:
        check(N.lib.infw_host_unregister(self._ctx, arr.ctypes.data), "host_unregister")

    def pack_frames(self, frames, linear_len, ifindex, out, pkt_len=None, offsets=None, stride: int = 0,
                    dev: int = 0, stream=None) -> None:
        """Frames in device memory (uint8 tensor) -> the SoA batch `out` on the device (§8f-3)."""
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(frames.device)
        sp = stream if isinstance(stream, int) else stream.cuda_stream
        fb = N.FrameBatch(frames.data_ptr(), offsets.data_ptr() if offsets is not None else None, stride,
                          linear_len.data_ptr(), pkt_len.data_ptr() if pkt_len is not None else None,
                          ifindex.data_ptr())
        o = N.BatchSoa(out.saddr.data_ptr(), out.ifindex.data_ptr(), out.pkt_len.data_ptr(), out.meta.data_ptr(),
                       out.l4word.data_ptr())
        check(N.lib.infw_pack_frames(self._ctx, dev, C.byref(fb), out.n, C.byref(o), sp), "pack_frames")

    def pack_frames_c(self, frames, linear_len, ifindex, out_c, pkt_len=None, offsets=None, stride: int = 0,
                      dev: int = 0, stream=None) -> None:
        """Frames in device memory -> the family-compact batch `out_c` (infw.batch.SoaBatchC) on the device."""
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(frames.device)
        sp = stream if isinstance(stream, int) else stream.cuda_stream
        fb = N.FrameBatch(frames.data_ptr(), offsets.data_ptr() if offsets is not None else None, stride,
                          linear_len.data_ptr(), pkt_len.data_ptr() if pkt_len is not None else None,
                          ifindex.data_ptr())
        o = N.BatchSoaC(out_c.saddr4.data_ptr(), out_c.v6tail.data_ptr(), out_c.ifindex.data_ptr(),
                        out_c.pkt_len.data_ptr(), out_c.meta.data_ptr(), out_c.l4word.data_ptr())
        check(N.lib.infw_pack_frames_c(self._ctx, dev, C.byref(fb), out_c.n, C.byref(o), sp), "pack_frames_c")

    def classify_frames(self, frames, linear_len, ifindex, n: int, results=None, verdicts=None, pkt_len=None,
                        offsets=None, stride: int = 0, dev: int = 0, stream=None, events=None, events_count=None) -> None:
        """infw_classify_frames: classify n frames in device memory (uint8 tensor) without a SoA batch — the same
        result words, verdicts and counters as pack_frames + classify.  events / events_count: the deny-event
        stream as in classify_events (infw_classify_frames_ex)."""
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(frames.device)
        sp = stream if isinstance(stream, int) else stream.cuda_stream
        fb = N.FrameBatch(frames.data_ptr(), offsets.data_ptr() if offsets is not None else None, stride,
                          linear_len.data_ptr(), pkt_len.data_ptr() if pkt_len is not None else None,
                          ifindex.data_ptr())
        ex = None
        if events is not None:
            ex = N.ClassifyEx(C.sizeof(N.ClassifyEx), 0, events.data_ptr(), events.numel() // C.sizeof(N.EventRec),
                              events_count.data_ptr())
        check(N.lib.infw_classify_frames_ex(self._ctx, dev, C.byref(fb), n,
                                            results.data_ptr() if results is not None else None,
                                            verdicts.data_ptr() if verdicts is not None else None,
                                            C.byref(ex) if ex is not None else None, sp), "classify_frames")

    def classify_xdp(self, umem, descs, n: int, ifindex: int, results=None, verdicts=None, dev: int = 0,
                     stream=None) -> None:
        """infw_classify_xdp: an AF_XDP RX ring's descriptors (`descs`: n x 16 B, struct xdp_desc) over the frames of
        `umem` — torch tensors in HBM or pinned host memory (read in place over PCIe); one ifindex for the ring.
        `results` / `verdicts` may be device or pinned host tensors."""
        if stream is None:
            import torch
            on = results.device if results is not None and results.is_cuda else torch.device("cuda", dev)
            stream = torch.cuda.current_stream(on)  # results / verdicts may be pinned host memory
        sp = stream if isinstance(stream, int) else stream.cuda_stream
        check(N.lib.infw_classify_xdp(self._ctx, dev, umem.data_ptr(), descs.data_ptr(), n, ifindex,
                                      results.data_ptr() if results is not None else None,
                                      verdicts.data_ptr() if verdicts is not None else None, sp), "classify_xdp")

    def classify_xdp_host(self, rings, chunk: int = 0, dev: int = 0) -> None:
        """infw_classify_xdp_host: AF_XDP RX rings over a host umem, packed on the context's host threads and
        classified through the device (synchronous).  `rings`: (umem, descs, n, ifindex, results, verdicts) per
        ring — host buffers as torch CPU tensors, numpy arrays or raw addresses; results / verdicts may be None."""
        def ptr(x):
            if x is None or isinstance(x, int):
                return x
            return x.data_ptr() if hasattr(x, "data_ptr") else x.ctypes.data
        arr = (N.XdpRing * max(1, len(rings)))()
        for i, (umem, descs, n, ifindex, results, verdicts) in enumerate(rings):
            arr[i] = N.XdpRing(ptr(umem), ptr(descs), n, ifindex, 0, ptr(results), ptr(verdicts))
        check(N.lib.infw_classify_xdp_host(self._ctx, dev, arr, len(rings), chunk), "classify_xdp_host")

    def classify_bursts_host(self, bursts, chunk: int = 0, dev: int = 0) -> None:
        """infw_classify_bursts_host (include/infw_host.h): DPDK-style bursts of frames in host memory — per burst a
        `Burst` (frame pointers, linear and frame lengths, ifindex, optional result / verdict arrays) — packed on the
        context's host threads and classified through the device (synchronous).  `bursts`: a list of Burst, or a
        BurstArray built once (the C array a daemon hands over; building it costs a few µs per burst in Python)."""
        arr = bursts if isinstance(bursts, BurstArray) else BurstArray(bursts)
        check(N.lib.infw_classify_bursts_host(self._ctx, dev, arr.arr, arr.n, chunk), "classify_bursts_host")

    def events_capture(self, frames, linear_len, ifindex, n_frames: int, events, events_count, samples,
                       pkt_len=None, offsets=None, stride: int = 0, dev: int = 0, stream=None) -> None:
        """The perf samples of the deny events classify_events wrote (kernel.c:392-399) from the frames the batch was
        packed from: `samples` is a uint8 tensor of (events capacity) x 272 B (infw_event_sample slots)."""
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(frames.device)
        sp = stream if isinstance(stream, int) else stream.cuda_stream
        fb = N.FrameBatch(frames.data_ptr(), offsets.data_ptr() if offsets is not None else None, stride,
                          linear_len.data_ptr(), pkt_len.data_ptr() if pkt_len is not None else None,
                          ifindex.data_ptr())
        cap = events.numel() // C.sizeof(N.EventRec)
        assert samples.numel() >= cap * N.EVENT_SAMPLE_BYTES, "samples: one 272-B slot per event record"
        check(N.lib.infw_events_capture(self._ctx, dev, C.byref(fb), n_frames, events.data_ptr(), cap,
                                        events_count.data_ptr(), samples.data_ptr(), sp), "events_capture")

    def set_launch(self, block: int = 768, scan_group: int = 0, blocks_per_cu: int = 2) -> None:
        """Launch shape of the classify kernel (tuning knob; see include/infw.h)."""
        check(N.lib.infw_set_launch(self._ctx, block, scan_group, blocks_per_cu), "set_launch")

    def launch(self) -> Tuple[int, int, int]:
        """(block, scan_group, blocks_per_cu) infw_classify launches with."""
        b, g, p = C.c_int(0), C.c_int(0), C.c_int(0)
        check(N.lib.infw_get_launch(self._ctx, C.byref(b), C.byref(g), C.byref(p)), "get_launch")
        return b.value, g.value, p.value

    # -- statistics map
    def _settle(self) -> None:
        """Wait for the work queued on this context's devices (torch streams included): the C readers take a
        snapshot without waiting for anything, like a per-CPU map read beside running XDP programs."""
        if self.num_devices:
            import torch
            for d in sorted(set(self._devices or [torch.cuda.current_device()])):
                torch.cuda.synchronize(d)

    def stats_read(self, rule_id: int, wait: bool = True) -> List[RuleStatisticsSt]:
        """Map.Lookup(uint32(rule), &[]BpfRuleStatisticsSt): one entry per device slot.  wait=False: the snapshot
        as the counters stand (what a poller beside running batches sees); True: after this process's queued work."""
        if wait:
            self._settle()
        nd = max(1, self.num_devices)
        arr = (RuleStatisticsSt * nd)()
        ns = C.c_int(0)
        check(N.lib.infw_stats_read(self._ctx, rule_id, arr, C.byref(ns)), "stats_read")
        return list(arr[: ns.value])

    def stats_read_all(self, wait: bool = True) -> np.ndarray:
        """All 1024 rules summed over slots (infw_stats_read_all); wait as for stats_read."""
        if wait:
            self._settle()
        arr = (RuleStatisticsSt * N.MAX_TARGETS)()
        check(N.lib.infw_stats_read_all(self._ctx, arr), "stats_read_all")
        return np.frombuffer(bytes(arr), dtype=np.uint64).reshape(N.MAX_TARGETS, 4).copy()

    def stats_reset(self) -> None:
        check(N.lib.infw_stats_reset(self._ctx), "stats_reset")

    def stats_bind(self, dev: int, ptr: Optional[int]) -> None:
        check(N.lib.infw_stats_bind(self._ctx, dev, ptr or None), "stats_bind")

    # -- debug lookup capture (ingress_node_firewall_dbg_map, kernel.c:59-64, :214-216, :297-299)
    def debug_lookup(self, value: int) -> None:
        """The debug_lookup load-time constant (loader.go:72-83): non-zero captures every lookup key."""
        check(N.lib.infw_debug_lookup_set(self._ctx, int(value)), "debug_lookup_set")

    def debug_keys(self) -> list:
        """Keys held by the debug map (union over devices), as 24-byte lpm_ip_key_st images."""
        arr = (LpmIpKeySt * N.DBG_MAX_ENTRIES)()
        n = C.c_uint32()
        check(N.lib.infw_debug_keys_read(self._ctx, arr, N.DBG_MAX_ENTRIES, C.byref(n)), "debug_keys_read")
        return [bytes(arr[i]) for i in range(min(n.value, N.DBG_MAX_ENTRIES))]

    def debug_keys_clear(self) -> None:
        check(N.lib.infw_debug_keys_clear(self._ctx), "debug_keys_clear")

    def stats_device_ptr(self, dev: int = 0) -> int:
        p = C.c_void_p()
        check(N.lib.infw_stats_device_ptr(self._ctx, dev, C.byref(p)), "stats_device_ptr")
        return p.value

    # -- verification hook (tests only)
    def debug_walk(self, tuples: np.ndarray) -> np.ndarray:
        t = np.ascontiguousarray(tuples, dtype=np.uint32).reshape(-1, 8)
        out = np.zeros(t.shape[0], dtype=np.uint32)
        check(N.lib.infw_debug_walk(self._ctx, t.ctypes.data, t.shape[0], out.ctypes.data), "debug_walk")
        return out


class HostSoa:
    """struct infw_batch_soa in host memory: five numpy streams (saddr n x 16 u8, ifindex, pkt_len, meta, l4word)."""

    def __init__(self, n: int):
        self.n = n
        self.saddr = np.zeros((n, 16), np.uint8)
        self.ifindex = np.zeros(n, np.uint32)
        self.pkt_len = np.zeros(n, np.uint32)
        self.meta = np.zeros(n, np.uint32)
        self.l4word = np.zeros(n, np.uint32)

    @staticmethod
    def from_tuples(t: np.ndarray) -> "HostSoa":
        """t: n x 8 u32 tuples {saddr[4], ifindex, pkt_len, meta, l4word}."""
        h = HostSoa(t.shape[0])
        h.saddr[:] = np.ascontiguousarray(t[:, :4]).view(np.uint8).reshape(-1, 16)
        h.ifindex[:], h.pkt_len[:], h.meta[:], h.l4word[:] = t[:, 4], t[:, 5], t[:, 6], t[:, 7]
        return h

    def arrays(self):
        return (self.saddr, self.ifindex, self.pkt_len, self.meta, self.l4word)

    def slice(self, a: int, b: int) -> "HostSoa":
        """Packets [a, b) as views of the same memory (no copy)."""
        h = HostSoa.__new__(HostSoa)
        h.n = b - a
        h.saddr, h.ifindex, h.pkt_len = self.saddr[a:b], self.ifindex[a:b], self.pkt_len[a:b]
        h.meta, h.l4word = self.meta[a:b], self.l4word[a:b]
        return h


class Burst:
    """struct infw_frame_burst: frames given as host addresses (uint64 array, e.g. rte_pktmbuf_mtod of each mbuf),
    their linear lengths (data_len) and frame lengths (pkt_len; None: the linear lengths), one ifindex; results /
    verdicts: numpy arrays to fill, or None.  Keeps its arrays alive while the C struct points at them."""

    def __init__(self, frames: np.ndarray, linear_len: np.ndarray, pkt_len: Optional[np.ndarray], ifindex: int,
                 results: Optional[np.ndarray] = None, verdicts: Optional[np.ndarray] = None):
        self.frames = np.ascontiguousarray(frames, np.uint64)
        self.linear_len = np.ascontiguousarray(linear_len, np.uint32)
        self.pkt_len = None if pkt_len is None else np.ascontiguousarray(pkt_len, np.uint32)
        self.n, self.ifindex, self.results, self.verdicts = self.frames.size, ifindex, results, verdicts

    def c(self) -> "N.FrameBurst":
        ptr = lambda a: None if a is None or a.size == 0 else a.ctypes.data  # noqa: E731
        return N.FrameBurst(ptr(self.frames), ptr(self.linear_len), ptr(self.pkt_len), self.n, self.ifindex, 0,
                            ptr(self.results), ptr(self.verdicts))


class BurstArray:
    """The struct infw_frame_burst array of a list of Burst, built once (keeps the bursts alive)."""

    def __init__(self, bursts):
        self.bursts = list(bursts)
        self.n = len(self.bursts)
        self.arr = (N.FrameBurst * max(1, self.n))()
        for i, b in enumerate(self.bursts):
            self.arr[i] = b.c()


def pack_burst_host(burst: Burst) -> Dict[str, np.ndarray]:
    """infw_pack_burst_host: a burst's frames -> the family-compact streams on the calling thread (numpy, host)."""
    n = burst.n
    out = {k: np.zeros(max(n, 1), np.uint32) for k in ("saddr4", "ifindex", "pkt_len", "meta", "l4word")}
    out["v6tail"] = np.zeros(max(1, (n + 63) // 64) * 768, np.uint8)
    o = N.BatchSoaC(*(out[k].ctypes.data for k in ("saddr4", "v6tail", "ifindex", "pkt_len", "meta", "l4word")))
    b = burst.c()
    check(N.lib.infw_pack_burst_host(C.byref(b), C.byref(o)), "pack_burst_host")
    return {k: v[:n] if k != "v6tail" else v for k, v in out.items()}


def burst_host_events(burst: Burst, results: np.ndarray, cap: int):
    """Deny-event perf samples of a burst from its result words (infw_burst_host_events): (cap x 272 uint8, count)."""
    r = np.ascontiguousarray(results, np.uint32)
    out = np.zeros((max(cap, 1), N.EVENT_SAMPLE_BYTES), np.uint8)
    k = C.c_uint64(0)
    b = burst.c()
    check(N.lib.infw_burst_host_events(C.byref(b), r.ctypes.data if r.size else None,
                                       out.ctypes.data if cap else None, cap, C.byref(k)), "burst_host_events")
    return out[:cap], k.value


def xdp_host_events(umem: np.ndarray, descs: np.ndarray, ifindex: int, results: np.ndarray, cap: int):
    """Deny-event perf samples of one AF_XDP ring from its frames and result words (infw_xdp_host_events,
    include/infw_host.h): (cap x 272 uint8 samples, events in the ring — also those past cap)."""
    n = descs.shape[0]
    d = np.ascontiguousarray(descs, np.uint32)
    r = np.ascontiguousarray(results, np.uint32)
    out = np.zeros((max(cap, 1), N.EVENT_SAMPLE_BYTES), np.uint8)
    k = C.c_uint64(0)
    check(N.lib.infw_xdp_host_events(umem.ctypes.data if n else None, d.ctypes.data if n else None, n, ifindex,
                                     r.ctypes.data if n else None, out.ctypes.data if cap else None, cap, C.byref(k)),
          "xdp_host_events")
    return out[:cap], k.value


def pack_xdp_host(umem: np.ndarray, descs: np.ndarray, ifindex: int) -> Dict[str, np.ndarray]:
    """infw_pack_xdp_host: the host packer of infw_classify_xdp_host on the calling thread — one AF_XDP ring's frames
    (`descs`: n x 16 B struct xdp_desc over the bytes of `umem`) -> the family-compact streams (numpy, host)."""
    descs = np.ascontiguousarray(descs).view(np.uint8).reshape(-1, 16)
    n = descs.shape[0]
    out = {k: np.zeros(max(n, 1), np.uint32) for k in ("saddr4", "ifindex", "pkt_len", "meta", "l4word")}
    out["v6tail"] = np.zeros(max(1, (n + 63) // 64) * 768, np.uint8)
    o = N.BatchSoaC(*(out[k].ctypes.data for k in ("saddr4", "v6tail", "ifindex", "pkt_len", "meta", "l4word")))
    umem = np.ascontiguousarray(umem)
    check(N.lib.infw_pack_xdp_host(umem.ctypes.data, descs.ctypes.data, n, ifindex, C.byref(o)), "pack_xdp_host")
    return {k: v[:n] if k != "v6tail" else v for k, v in out.items()}


def compact_to_tuples(c: Dict[str, np.ndarray]) -> np.ndarray:
    """Family-compact streams -> n x 8 u32 tuples {saddr[4], ifindex, pkt_len, meta, l4word} (infw_debug_walk's input;
    the inverse of the compact layout: a group's IPv6 packets take its tail slots in packet order)."""
    n = c["meta"].shape[0]
    t = np.zeros((n, 8), np.uint32)
    t[:, 0] = c["saddr4"]
    tails = c["v6tail"].view(np.uint32)
    is6 = (c["meta"] & 0xFFFF) == 0x86DD
    for g in range(0, n, 64):
        idx = np.nonzero(is6[g:g + 64])[0] + g
        base = g // 64 * 192
        for r, i in enumerate(idx):
            t[i, 1:4] = tails[base + 3 * r: base + 3 * r + 3]
    t[:, 4], t[:, 5], t[:, 6], t[:, 7] = c["ifindex"], c["pkt_len"], c["meta"], c["l4word"]
    return t


def verdicts_from_results(results: np.ndarray, meta: np.ndarray) -> np.ndarray:
    """XDP verdict implied by a result word (kernel.c:423-456)."""
    cap = (meta >> 24) & 0xFF
    act = results & 0xFF
    return np.where((cap < 14) | (act == N.XDP_DROP), N.XDP_DROP, N.XDP_PASS).astype(np.uint8)
