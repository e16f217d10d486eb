"""An AF_XDP RX ring as the feed (infw_classify_xdp): descriptors {addr, len, options} as the kernel
writes them into the ring (linux/if_xdp.h struct xdp_desc) over frames in a umem of 2048-B chunks, in aligned mode
(frames at chunk + headroom, chunks handed out in a shuffled order, as a fill ring recycles them) and in unaligned mode
(the offset in address bits 48..63).  The umem and the ring live in HBM or in pinned host memory, which the kernel
reads in place over PCIe.  Result words, verdicts and per-rule counters must equal the oracle's on the same frames
(single-buffer frames: the descriptor length is the linear length and the frame length; one ifindex per ring)."""
import numpy as np
import pytest
import torch

import infw
from infw import workloads as W

from parity import oracle_for

pytestmark = pytest.mark.gpu
CHUNK, HEADROOM = 2048, 256


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _ring(hdr, pl, mode, rng):
    """umem bytes and descriptors for the frames: aligned (chunk + headroom, shuffled chunks) or unaligned."""
    n = hdr.shape[0]
    chunks = rng.permutation(n + 7)[:n]
    umem = np.zeros((n + 7) * CHUNK, np.uint8)
    desc = np.zeros((n, 4), np.uint32)
    for i in range(n):
        if mode == "aligned":
            base, off = int(chunks[i]) * CHUNK + HEADROOM, 0
        else:  # unaligned: base address in bits 0..47, offset in 48..63, frame at base + offset
            base, off = int(chunks[i]) * CHUNK, int(rng.integers(0, CHUNK - 96))
        at = base + off
        umem[at:at + hdr.shape[1]] = hdr[i]
        addr = base | (off << 48)
        desc[i, 0], desc[i, 1], desc[i, 2] = addr & 0xFFFFFFFF, addr >> 32, pl[i]
    return umem, desc


@pytest.mark.parametrize("where", ["hbm", "host"])
@pytest.mark.parametrize("mode", ["aligned", "unaligned"])
def test_xdp_ring_matches_oracle(where, mode):
    rng = np.random.default_rng(7)
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=50000, n_templates=256)
    n, start = (1 << 15) + 77, 12345
    hdr, cap, pl, ifx = wl.frames(start, n)
    ring_if = int(np.bincount(ifx).argmax())  # one interface queue: every frame of the ring arrives on it
    ifx_all = np.full(n, ring_if, np.uint32)
    m = oracle_for(wl)
    want, wver, wst, _ = m.classify_frames(hdr, pl.astype(cap.dtype), pl, ifx_all, nthreads=8)
    umem, desc = _ring(hdr, pl, mode, rng)
    dev = torch.device("cuda", 0)
    if where == "hbm":
        tu, td = torch.from_numpy(umem).to(dev), torch.from_numpy(desc.view(np.int32)).to(dev)
    else:  # pinned host memory: the kernel reads the umem and the ring over PCIe
        tu = torch.from_numpy(umem).pin_memory()
        td = torch.from_numpy(desc.view(np.int32)).pin_memory()
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    res = torch.empty(n, dtype=torch.int32, device=dev)
    ver = torch.empty(n, dtype=torch.uint8, device=dev)
    clf.stats_reset()
    clf.classify_xdp(tu, td, n, ring_if, results=res, verdicts=ver)
    torch.cuda.synchronize()
    got = res.cpu().numpy().view(np.uint32)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (where, mode, bad[:5], got[bad[:5]], want[bad[:5]])
    assert np.array_equal(ver.cpu().numpy(), wver)
    assert np.array_equal(clf.stats_read_all(), wst)
    assert (want & 0xFF).astype(bool).mean() > 0.3  # the frames exercise the rules


def test_xdp_results_in_host_memory():
    """A daemon may take the verdicts straight into pinned host memory: umem, ring, result
    words and verdicts all in pinned host memory, the kernel reading and writing over PCIe."""
    rng = np.random.default_rng(11)
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=20000, n_templates=64)
    n = (1 << 13) + 5
    hdr, cap, pl, ifx = wl.frames(777, n)
    ring_if = int(np.bincount(ifx).argmax())
    want, wver, wst, _ = oracle_for(wl).classify_frames(hdr, pl.astype(cap.dtype), pl, np.full(n, ring_if, np.uint32),
                                                        nthreads=8)
    umem, desc = _ring(hdr, pl, "aligned", rng)
    tu = torch.from_numpy(umem).pin_memory()
    td = torch.from_numpy(desc.view(np.int32)).pin_memory()
    res = torch.full((n,), -1, dtype=torch.int32).pin_memory()
    ver = torch.full((n,), 7, dtype=torch.uint8).pin_memory()
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 16)
    wl.load_into(clf)
    clf.commit()
    clf.stats_reset()
    clf.classify_xdp(tu, td, n, ring_if, results=res, verdicts=ver)
    torch.cuda.synchronize()
    assert np.array_equal(res.numpy().view(np.uint32), want)
    assert np.array_equal(ver.numpy(), wver)
    assert np.array_equal(clf.stats_read_all(), wst)


def test_xdp_rejects_bad_arguments():
    clf = infw.Classifier(devices=[0])
    dev = torch.device("cuda", 0)
    umem = torch.zeros(4096, dtype=torch.uint8, device=dev)
    desc = torch.zeros(12, dtype=torch.int32, device=dev)
    res = torch.empty(2, dtype=torch.int32, device=dev)
    with pytest.raises(infw.InfwError) as e:  # descriptors not 16-byte aligned
        clf.classify_xdp(umem, desc[1:], 2, 1, results=res)
    assert e.value.errno == 22
    clf.classify_xdp(umem, desc, 0, 1, results=res)  # an empty ring is a no-op
