"""SoA packet batches (include/infw.h: infw_batch_soa) held in torch device memory.

torch is used here for device allocation and copies only; the classifier
never sees torch types (it gets raw device pointers).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass
class SoaBatch:
    saddr: "torch.Tensor"    # uint8 [n, 16], 16-B aligned
    ifindex: "torch.Tensor"  # int32 [n] (u32 bits)
    pkt_len: "torch.Tensor"  # int32 [n]
    meta: "torch.Tensor"     # int32 [n]
    l4word: "torch.Tensor"   # int32 [n]

    @property
    def n(self) -> int:
        return int(self.ifindex.shape[0])

    @property
    def device(self):
        return self.ifindex.device

    @staticmethod
    def empty(n: int, device) -> "SoaBatch":
        import torch
        return SoaBatch(torch.empty((n, 16), dtype=torch.uint8, device=device),
                        torch.empty(n, dtype=torch.int32, device=device),
                        torch.empty(n, dtype=torch.int32, device=device),
                        torch.empty(n, dtype=torch.int32, device=device),
                        torch.empty(n, dtype=torch.int32, device=device))

    @staticmethod
    def from_tuples(tuples: np.ndarray, device) -> "SoaBatch":
        """tuples: n x 8 u32 {saddr[4], ifindex, pkt_len, meta, l4word} (host) -> device SoA."""
        import torch
        t = np.ascontiguousarray(tuples, dtype=np.uint32).reshape(-1, 8)
        sa = np.ascontiguousarray(t[:, 0:4]).view(np.uint8).reshape(-1, 16)
        col = lambda j: torch.from_numpy(np.ascontiguousarray(t[:, j]).view(np.int32)).to(device)
        return SoaBatch(torch.from_numpy(sa).to(device), col(4), col(5), col(6), col(7))

    def to_tuples(self) -> np.ndarray:
        n = self.n
        out = np.empty((n, 8), dtype=np.uint32)
        out[:, 0:4] = self.saddr.cpu().numpy().view(np.uint32).reshape(n, 4)
        for j, t in ((4, self.ifindex), (5, self.pkt_len), (6, self.meta), (7, self.l4word)):
            out[:, j] = t.cpu().numpy().view(np.uint32)
        return out

    def slice(self, a: int, b: int) -> "SoaBatch":
        return SoaBatch(self.saddr[a:b], self.ifindex[a:b], self.pkt_len[a:b], self.meta[a:b], self.l4word[a:b])


@dataclass
class SoaBatchC:
    """Family-compact layout (include/infw.h: infw_batch_soa_c): 4 address bytes per packet plus, per group
    of 64 packets, the IPv6 packets' remaining 12 bytes packed at the front of a 768-B block.  The other
    streams are the standard batch's tensors (shared, not copied)."""
    saddr4: "torch.Tensor"   # int32 [n]
    v6tail: "torch.Tensor"   # uint8 [ceil(n / 64) * 768]
    ifindex: "torch.Tensor"
    pkt_len: "torch.Tensor"
    meta: "torch.Tensor"
    l4word: "torch.Tensor"

    @property
    def n(self) -> int:
        return int(self.ifindex.shape[0])

    @property
    def device(self):
        return self.ifindex.device

    @staticmethod
    def empty(n: int, device) -> "SoaBatchC":
        import torch
        i32 = lambda: torch.empty(n, dtype=torch.int32, device=device)
        return SoaBatchC(i32(), torch.zeros(((n + 63) // 64) * 768, dtype=torch.uint8, device=device), i32(), i32(),
                         i32(), i32())

    @staticmethod
    def empty_for(b: SoaBatch) -> "SoaBatchC":
        import torch
        groups = (b.n + 63) // 64
        return SoaBatchC(torch.empty(b.n, dtype=torch.int32, device=b.device),
                         torch.zeros(groups * 768, dtype=torch.uint8, device=b.device),
                         b.ifindex, b.pkt_len, b.meta, b.l4word)
