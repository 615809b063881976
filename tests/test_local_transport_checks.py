"""The in-process transport's schedule checks (include/gdf_fused.h gdf_fused_local_check_round /
_check_arrival: what every round of gdf_fused_local verifies on every rank before any copy), fired
on deliberately bad schedules.  No GPU: the checks read the posted operations (addresses are
compared, never dereferenced).

Each bad schedule is one RCCL would hang on or corrupt: a send no peer receives (the sender's
kernel never completes), a receive without its send, sizes that differ, an all-gather whose send
buffer overlaps its receive buffer other than at recv + rank * bytes (RCCL's only in-place form),
and ranks issuing the two communicators' collectives in different orders (the two-communicator
deadlock)."""
import ctypes as C

import pytest

AG, SEND, RECV = 0, 1, 2
HALO, POINTS = 0, 1


def lib():
    from ros_gpu_depthmap_fusion_amd import build_library
    from ros_gpu_depthmap_fusion_amd.gdf import load_library
    build_library()
    return load_library()


def check_round(per_rank, issue=None):
    """per_rank[q] = [(kind, src, dst, bytes, peer), ...]; returns (rc, message)."""
    from ros_gpu_depthmap_fusion_amd.gdf import LocalOp
    L = lib()
    W = len(per_rank)
    flat = [op for ops in per_rank for op in ops]
    arr = (LocalOp * max(len(flat), 1))()
    for j, (k, s, d, b, p) in enumerate(flat):
        arr[j].kind, arr[j].src, arr[j].dst, arr[j].bytes, arr[j].peer = k, s, d, b, p
    nops = (C.c_uint32 * W)(*[len(ops) for ops in per_rank])
    iss = (C.c_uint64 * W)(*(issue or [5] * W))
    rc = L.gdf_fused_local_check_round(W, arr, nops, iss)
    return rc, L.gdf_last_error().decode()


def ring_exchange(W, nbytes=64):
    """rank q sends nbytes to q + 1 and receives from q - 1 (distinct fake addresses)."""
    return [[(SEND, 0x10000 * (q + 1), None, nbytes, (q + 1) % W),
             (RECV, None, 0x10000 * (q + 1) + 0x8000, nbytes, (q - 1) % W)] for q in range(W)]


def test_valid_schedules_pass():
    assert check_round(ring_exchange(3))[0] == 0
    # in-place all-gather (send = recv + rank * bytes), then a disjoint one
    b = 256
    rounds = [[(AG, 0x100000 * (q + 1) + q * b, 0x100000 * (q + 1), b, -1),
               (AG, 0x900000 + q * 0x1000, 0x200000 * (q + 1), b, -1)] for q in range(4)]
    assert check_round(rounds)[0] == 0
    # the step's points group: per peer, three sends and three receives in the same order
    W = 3
    grp = []
    for q in range(W):
        ops = []
        for r in range(W):
            if r == q:
                continue
            for k, nb in enumerate((160, 40, 40)):
                ops.append((SEND, 0x1000 * (10 * q + k + 1), None, nb, r))
            for k, nb in enumerate((160, 40, 40)):
                ops.append((RECV, None, 0x1000 * (100 + 10 * q + k), nb, r))
        grp.append(ops)
    assert check_round(grp)[0] == 0


def test_send_no_receive_consumes_fails():
    s = ring_exchange(3)
    s[1] = [op for op in s[1] if op[0] != RECV]  # rank 1 never receives rank 0's send
    rc, msg = check_round(s)
    assert rc == -2 and "a send no receive consumes (rank 0 -> rank 1)" in msg, msg


def test_receive_without_send_fails():
    s = ring_exchange(3)
    s[2] = [op for op in s[2] if op[0] != SEND]  # rank 0 waits for rank 2's send
    rc, msg = check_round(s)
    assert rc == -2 and "a receive without its send (rank 2 -> rank 0)" in msg, msg


def test_send_receive_sizes_differ_fails():
    s = ring_exchange(2)
    k, src, dst, b, p = s[0][0]
    s[0][0] = (k, src, dst, b + 4, p)
    rc, msg = check_round(s)
    assert rc == -2 and "send / receive sizes differ" in msg, msg


def test_bad_peer_fails():
    s = ring_exchange(2)
    s[0][0] = (SEND, 0x1000, None, 64, 0)  # to itself
    assert "bad send peer" in check_round(s)[1]
    s = ring_exchange(2)
    s[1][1] = (RECV, None, 0x2000, 64, 7)
    assert "bad receive peer" in check_round(s)[1]


@pytest.mark.parametrize("src_of", [
    lambda dst, q, b: dst,                # every rank sends from slot 0
    lambda dst, q, b: dst + q * b + 8,    # misaligned inside its own slot
    lambda dst, q, b: dst + 4 * b - 16,   # straddles the receive buffer's end
])
def test_all_gather_illegal_in_place_fails(src_of):
    b, W = 256, 4
    s = [[(AG, src_of(0x100000 * (q + 1), q, b), 0x100000 * (q + 1), b, -1)] for q in range(W)]
    rc, msg = check_round(s)
    # rank 0's slot is its own buffer start: only the ranks with q > 0 (or a straddle) fail
    assert rc == -2 and "overlaps its receive buffer other than at recv + rank * bytes" in msg, msg


def test_all_gather_sizes_differ_fails():
    s = [[(AG, 0x10000 * q, 0x900000 + 0x10000 * q, 64 if q else 128, -1)] for q in range(2)]
    rc, msg = check_round(s)
    assert rc == -2 and "all-gather sizes differ" in msg, msg
    s = [[(AG, 0x10000 * q, 0x900000 + 0x10000 * q, 64, -1)] * (1 + q) for q in range(2)]
    assert "all-gather sizes differ" in check_round(s)[1]


def test_issue_numbers_differ_fails():
    rc, msg = check_round(ring_exchange(3), issue=[7, 7, 8])
    assert rc == -2 and "cross-communicator issue order differs" in msg, msg


def check_arrival(W, rank, comm, rnd, issue, waiting):
    L = lib()
    flat = []
    for w in waiting:
        flat += list(w) if w else [-1, -1, -1]
    arr = (C.c_int64 * (3 * W))(*flat)
    rc = L.gdf_fused_local_check_arrival(W, rank, comm, rnd, issue, arr)
    return rc, L.gdf_last_error().decode()


def test_crossed_communicators_fail_on_arrival():
    """Rank 0 issued the halo round 4 as its collective #9 and waits in it; rank 1 issues the
    points round 3 as #9: the ranks' orders crossed (each would wait for the other for ever)."""
    rc, msg = check_arrival(2, 1, POINTS, 3, 9, [(HALO, 4, 9), None])
    assert rc == -2 and "cross-communicator issue order differs" in msg and "halo round 4" in msg, msg
    # the same round under the same number, or another round under another number: fine
    assert check_arrival(2, 1, POINTS, 3, 9, [(POINTS, 3, 9), None])[0] == 0
    assert check_arrival(3, 2, HALO, 5, 11, [(POINTS, 4, 10), None, None])[0] == 0
    assert check_arrival(3, 0, HALO, 5, 11, [None, None, None])[0] == 0


def test_check_arguments():
    L = lib()
    assert L.gdf_fused_local_check_round(0, None, None, None) == -1
    assert L.gdf_fused_local_check_arrival(2, 2, 0, 0, 0, (C.c_int64 * 6)()) == -1
