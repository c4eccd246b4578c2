"""Quorum tally kernel vs the reference voter-set semantics."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_tally_fixture(tally_fx):
    from plenum_gpu.models import tally_batches
    t = tally_fx
    votes, reached = tally_batches(t['verdict'], t['sender'], t['batch_off'], int(t['n_nodes']),
                                   int(t['commit_quorum']))
    assert (votes == t['vote_count']).all()
    assert (reached == t['commit_reached'].astype(bool)).all()
    _, reached_p = tally_batches(t['verdict'], t['sender'], t['batch_off'], int(t['n_nodes']),
                                 int(t['prepare_quorum']))
    assert (reached_p == t['prepare_reached'].astype(bool)).all()


@pytest.mark.parametrize('n_nodes', [4, 25, 64, 65, 200, 1024])
def test_tally_random_vs_sets(n_nodes):
    from plenum_gpu.models import Commits, tally_batches
    from plenum_gpu.quorums import Quorums
    rng = np.random.default_rng(n_nodes)
    nb = 700
    sizes = rng.integers(0, 2 * n_nodes + 3, nb)
    off = np.zeros(nb + 1, np.uint64)
    off[1:] = np.cumsum(sizes)
    m = int(off[-1])
    sender = rng.integers(0, n_nodes, m).astype(np.uint32)
    verdict = rng.random(m) < 0.8
    q = Quorums(n_nodes).commit.value
    votes, reached = tally_batches(verdict, sender, off, n_nodes, q)

    class C:
        def __init__(self, b):
            self.viewNo, self.ppSeqNo = 0, b
    commits = Commits()
    for b in range(nb):
        c = C(b)
        for k in range(int(off[b]), int(off[b + 1])):
            if verdict[k]:
                commits.addVote(c, 'Node%d' % sender[k])
        assert votes[b] == commits._votes_count(c)
        assert reached[b] == commits.hasQuorum(c, q)


def test_propagate_fixture_gpu():
    """Row f4 pinned to the reference: the PROPAGATE streams of
    tests/golden/propagate.json (reference Requests store + Quorums(n).propagate,
    re-sent / duplicate / non-str senders, tampered and re-signed requests).
    Signature verdicts come from THIS engine (ReqAuthenticator.verify_batch on
    the GPU), the voter sets from the GPU tally."""
    import _propagate_cases as pc
    from plenum_gpu.client_authn import CoreAuthNr
    from plenum_gpu.ingress import request_key
    from plenum_gpu.models import propagate_quorums
    from plenum_gpu.req_authenticator import ReqAuthenticator
    fx = pc.load()
    authnr = CoreAuthNr(fx['write_types'], [], [])
    for idr, vk in fx['registry'].items():
        authnr.addIdr(idr, vk)
    ra = ReqAuthenticator()
    ra.register_authenticator(authnr)
    reqs = [c['req'] for c in fx['cases']]
    keys = [request_key(r) for r in reqs]
    assert keys == [c['key'] for c in fx['cases']]
    res = ra.verify_batch(reqs, keys)
    valid = [not isinstance(r, BaseException) for r in res]
    assert valid == [c['valid'] for c in fx['cases']]
    for st in fx['streams']:
        got = propagate_quorums(*pc.stream_arrays(fx, st, valid), st['n'])
        assert list(got) == st['order']
        for key, want in st['outcome'].items():
            g = got[key]
            assert (g.votes, g.reached, g.finalised_by) == (want['str_votes'], want['reached'],
                                                            want['finalised_by']), (st['n'], key)
            if g.reached:
                snd, ci = st['events'][g.event]
                assert snd == want['finalised_by'] and fx['cases'][ci]['key'] == key


def test_tally_bitmap_form_fixture(tally_fx):
    """SURVEY.md §8(b) pv_tally (node-indexed voter bitmaps + dup mask) on the
    reference-generated COMMIT batches of tally.npz."""
    from plenum_gpu import _native as nat
    t = tally_fx
    n = int(t['n_nodes'])
    off = t['batch_off'].astype(np.int64)
    nb = len(off) - 1
    bits = np.zeros((nb, (n + 31) // 32), np.uint32)
    for b in range(nb):
        for k in range(off[b], off[b + 1]):
            if t['verdict'][k]:
                s = int(t['sender'][k])
                bits[b, s // 32] |= np.uint32(1 << (s % 32))
    assert (nat.tally_bits_arrays(bits, n, int(t['commit_quorum'])) == t['commit_reached'].astype(bool)).all()
    assert (nat.tally_bits_arrays(bits, n, int(t['prepare_quorum'])) == t['prepare_reached'].astype(bool)).all()
    # masking node 0 out of every batch = the reference count without node 0's votes
    dup = np.zeros_like(bits)
    dup[:, 0] = 1
    want = [sum(1 for s in set(int(t['sender'][k]) for k in range(off[b], off[b + 1]) if t['verdict'][k]) if s)
            >= int(t['commit_quorum']) for b in range(nb)]
    assert (nat.tally_bits_arrays(bits, n, int(t['commit_quorum']), dup_mask=dup) == np.array(want)).all()


@pytest.mark.parametrize('n_nodes', [1, 31, 32, 33, 100])
def test_tally_bitmap_random(n_nodes):
    from plenum_gpu import _native as nat
    rng = np.random.default_rng(n_nodes)
    w = (n_nodes + 31) // 32
    bits = rng.integers(0, 2 ** 32, (500, w), dtype=np.uint64).astype(np.uint32)
    dup = (rng.integers(0, 2 ** 32, (500, w), dtype=np.uint64) & rng.integers(0, 2 ** 32, (500, w),
                                                                                 dtype=np.uint64)).astype(np.uint32)
    q = max(1, (2 * n_nodes) // 3)
    got = nat.tally_bits_arrays(bits, n_nodes, q, dup_mask=dup)
    for b in range(500):
        cnt = sum(1 for j in range(n_nodes) if (int(bits[b, j // 32]) >> (j % 32)) & 1
                  and not (int(dup[b, j // 32]) >> (j % 32)) & 1)
        assert got[b] == (cnt >= q)


def test_tally_rejects_out_of_range_sender():
    from plenum_gpu import _native as nat
    from plenum_gpu.models import tally_batches
    with pytest.raises(nat.PlenumGpuError, match='n_nodes'):
        tally_batches([1, 1], [0, 25], [0, 2], 25, 1)


def test_tally_device_rejects_out_of_range_sender():
    import torch
    from plenum_gpu import _native as nat
    from plenum_gpu.device import tally_device
    dev = torch.device('cuda:0')
    v = torch.ones(2, dtype=torch.uint8, device=dev)
    s = torch.tensor([0, 25], dtype=torch.int32, device=dev)
    off = torch.tensor([0, 2], dtype=torch.int64, device=dev)
    votes = torch.zeros(1, dtype=torch.int32, device=dev)
    reached = torch.zeros(1, dtype=torch.uint8, device=dev)
    with pytest.raises(nat.PlenumGpuError, match='n_nodes'):
        tally_device(v, s, off, 25, 1, votes, reached)
    s[1] = 24
    tally_device(v, s, off, 25, 2, votes, reached)
    assert int(votes[0]) == 2 and int(reached[0]) == 1


def test_tally_device_async_flag_and_side_stream():
    """pv_tally_votes_device_async: enqueue-only on a side stream, same tallies
    as the synchronous form; an out-of-range sender raises the device flag
    (and is not counted) instead of failing the call."""
    import torch
    from plenum_gpu.device import tally_device, tally_device_async
    dev = torch.device('cuda:0')
    g = torch.Generator().manual_seed(7)
    nb, nn = 1000, 25
    v = (torch.rand(nb * nn, generator=g) > 0.2).to(torch.uint8).to(dev)
    s = torch.randint(0, nn, (nb * nn,), generator=g, dtype=torch.int32).to(dev)
    off = (torch.arange(nb + 1, dtype=torch.int64) * nn).to(dev)
    want_v = torch.empty(nb, dtype=torch.int32, device=dev)
    want_r = torch.empty(nb, dtype=torch.uint8, device=dev)
    tally_device(v, s, off, nn, 17, want_v, want_r)
    votes = torch.empty(nb, dtype=torch.int32, device=dev)
    reached = torch.empty(nb, dtype=torch.uint8, device=dev)
    bad = torch.zeros(1, dtype=torch.int32, device=dev)
    st = torch.cuda.Stream(dev)
    st.wait_stream(torch.cuda.current_stream(dev))
    tally_device_async(v, s, off, nn, 17, votes, reached, bad, st)
    st.synchronize()
    assert int(bad[0]) == 0
    assert torch.equal(votes, want_v) and torch.equal(reached, want_r)
    s[3] = nn
    tally_device_async(v, s, off, nn, 17, votes, reached, bad)
    torch.cuda.synchronize()
    assert int(bad[0]) != 0
    # the out-of-range vote is dropped: batch 0 counts the distinct valid senders left
    vh, sh = v[:nn].cpu().tolist(), s[:nn].cpu().tolist()
    assert int(votes[0]) == len({sh[m] for m in range(nn) if vh[m] and sh[m] < nn})
    assert torch.equal(votes[1:], want_v[1:])
