"""The C ABI's threading contract on the device (include/infw.h "threads"): the reference's syncer edits and reloads
the maps under e.mu while XDP keeps classifying on every CPU (pkg/ebpfsyncer/ebpfsyncer.go:62, 72-73).  Here one host
thread classifies a fixed batch in a loop on its own stream while a second thread applies a sequence of edit sets
through the map API and commits each — incremental commits that patch the spare device image while batches run on
the live one.  Every batch's result words must equal exactly one epoch's oracle output (each batch sees one committed
epoch), the epochs seen must not go backwards, and the device counters must equal the sum of the oracle counters of
the epochs the batches saw.  (The host-side form under ThreadSanitizer: tests/test_threads_cpu.py.)"""
import random
import threading
import time

import numpy as np
import pytest
import torch

import infw
from infw import workloads as W
from infw.batch import SoaBatch
from parity import oracle_for

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def test_classify_thread_beside_commit_thread():
    rng = random.Random(41)
    wl = W.Workload(W.CFG2_MIXED_1M, n_prefixes=50000, n_templates=256)
    ents = list(wl.entries())          # the generator's popularity order: the hot keys first
    hot = [k for k, _ in ents[:3000]]
    tmpl = sorted({v for _, v in ents})
    m = oracle_for(wl)
    n, start = 1 << 18, 777
    hdr, cap, pl, ifx = wl.frames(start, n)
    # the epochs: 0 = the workload, e = e-1 + 400 rewrites, 100 deletes, 100 re-adds of hot keys
    live = dict(ents)
    edits = [[]]
    for e in range(1, 7):
        es = []
        for _ in range(400):
            es.append((rng.choice(hot), rng.choice(tmpl)))
        for _ in range(100):
            k = rng.choice(hot)
            es.append((k, None))
        for _ in range(100):
            es.append((rng.choice(hot), rng.choice(tmpl)))
        edits.append(es)
    want = []
    for e, es in enumerate(edits):
        for k, v in es:
            if v is None:
                if k in live:
                    del live[k]
                    assert m.delete(k) == 0
            else:
                live[k] = v
                assert m.update(k, v) == 0
        ores, _, ost, _ = m.classify_frames(hdr, cap, pl, ifx, nthreads=8)
        want.append((ores, ost))
    assert len({w[0].tobytes() for w in want}) == len(want), "every epoch must classify the batch differently"

    dev = torch.device("cuda", 0)
    clf = infw.Classifier(devices=[0], max_entries=wl.n_entries + 4096)
    wl.load_into(clf)
    clf.commit()
    batch = SoaBatch.empty(n, dev)
    wl.gen_device(batch, start, 0)
    torch.cuda.synchronize()
    clf.stats_reset()
    seen, stop, errors = [], threading.Event(), []

    def classifier():
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream(dev)
            res = torch.empty(n, dtype=torch.int32, device=dev)
            after = 0
            while after < 3:
                clf.classify(batch, results=res, stream=s)
                s.synchronize()
                seen.append(res.cpu().numpy().view(np.uint32).copy())
                after += stop.is_set()
        except BaseException as e:
            errors.append(e)

    def syncer():
        try:
            live2 = {k for k, _ in ents}
            for es in edits[1:]:
                for k, v in es:
                    key = infw.LpmIpKeySt.from_buffer_copy(k)
                    if v is None:
                        if k in live2:
                            clf.delete(key)
                            live2.discard(k)
                    else:
                        clf.update(key, infw.RulesValSt.from_buffer_copy(v))
                        live2.add(k)
                clf.commit()
                assert clf.info()["commit_mode"] == infw.COMMIT_INCREMENTAL, clf.info()["full_reason"]
                time.sleep(0.01)
        except BaseException as e:
            errors.append(e)
        finally:
            stop.set()

    th = [threading.Thread(target=classifier), threading.Thread(target=syncer)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    assert not errors, errors[0]
    keys = {w[0].tobytes(): e for e, w in enumerate(want)}
    epochs = []
    for r in seen:
        e = keys.get(r.tobytes())
        assert e is not None, "a batch's results match no single epoch"
        epochs.append(e)
    assert epochs == sorted(epochs), "a batch saw an older epoch after a newer one"
    assert epochs[-1] == len(want) - 1 and len(set(epochs)) >= 2, epochs
    expect = np.zeros((1024, 4), np.uint64)
    for e in epochs:
        expect += want[e][1]
    assert np.array_equal(clf.stats_read_all(), expect)
