"""Device-output getitem batches of >= 4096 keys take the overlapped path (host key
lookups for the tail run while k_decode expands the head; the tail launches on a
second stream).  Its offsets, lengths, statuses and bytes must equal the plain path's
(host output, lookups first) on the same store, with missing and repeated keys mixed
in, and a too-small output buffer must report PX_ESPACE with the same `needed`."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
px = pytest.importorskip("pixiu_amd")


def _keys(cp, n, rng):
    keys = [cp.key(i) for i in range(n)]
    # missing keys, a key prefix, repeats: spread through head and tail
    extra = [b"no-such-key-%d" % i for i in range(40)] + [cp.key(3)[:-1], cp.key(5), cp.key(n - 1)]
    for k in extra:
        keys.insert(int(rng.integers(0, len(keys) + 1)), k)
    return keys


@pytest.mark.parametrize("rps", [2, 16])
def test_overlapped_equals_plain(rps):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from pixiu_amd import synth
    n = 5000
    cp = synth.make(3, n)
    rng = np.random.default_rng(7)
    keys = _keys(cp, n, rng)
    kb, ko = px.csr(keys)
    with px.Store(records_per_shard=rps) as st:
        r = st.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
        assert int(r["status"].max()) == 0
        want = st.get_batch((kb, ko), px.COMPAT)  # host output: plain path
        cap = int(2 * cp.raw_bytes + 256 * len(keys) + (1 << 20))
        out = torch.empty(cap, dtype=torch.uint8, device="cuda")
        rc, off, ln, sts, need = st.get_batch_device((kb, ko), out.data_ptr(), cap, px.COMPAT)
        assert rc == px.PX_ENOTFOUND  # the missing keys
        host = out.cpu().numpy()
        for i, w in enumerate(want):
            if w is None:
                assert sts[i] == px.PX_ENOTFOUND and ln[i] == 0
            else:
                assert sts[i] == px.PX_OK
                assert host[int(off[i]):int(off[i]) + int(ln[i])].tobytes() == w, f"key {i}"
        # offsets are the plain path's: each found key's slot is doc_len + 64 rounded to 16
        assert int(off[0]) == 0 and np.all(np.diff(off.astype(np.int64)) >= 0)
        # too small: PX_ESPACE with the same requirement, whether the head fits or not
        for small in (need - 1, 1 << 16):
            rc2, _, _, _, need2 = st.get_batch_device((kb, ko), out.data_ptr(), int(small), px.COMPAT)
            assert rc2 == px.PX_ESPACE and need2 == need
    # the plain path on device output (decode_waves pinned) agrees too
    with px.Store(records_per_shard=rps, decode_waves=4096) as st2:
        st2.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
        out2 = torch.empty(cap, dtype=torch.uint8, device="cuda")
        rc3, off3, ln3, sts3, need3 = st2.get_batch_device((kb, ko), out2.data_ptr(), cap, px.COMPAT)
        assert rc3 == rc and need3 == need
        assert np.array_equal(off3, off) and np.array_equal(ln3, ln) and np.array_equal(sts3, sts)
        host2 = out2.cpu().numpy()
        for i in range(len(keys)):
            a, b = int(off[i]), int(off[i]) + int(ln[i])
            assert host2[a:b].tobytes() == host[a:b].tobytes(), f"key {i}"
