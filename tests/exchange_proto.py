"""The multi-GPU member step's exchange block, restated in numpy (test
infrastructure): what one rank ships in the all-gather of csrc/phj_group.h.

The library's own host-only ABI defines the rules (phj_exchange_geometry:
which digit of a hash code groups the block -- the LDS join's clusters or
the code tables' final partitions; phj_exchange_layout: codes | padding |
bounds). This module packs a rank's R shard by those rules from the oracle's
hash codes, reads gathered blocks back as segments, and compares a block
with another as the protocol allows: bounds exact, each segment's codes the
same multiset (the device pass leaves the order inside a segment free).
"""
import numpy as np

import partitionedhashjoin_amd as phj
from oracle import oracle as O


def geometry(params, total_build):
    """(num_segments, segment_of(codes) -> segment indices)."""
    nseg, shift, sub_bits, sub_shift, _cluster = phj.exchange_geometry(params, total_build)
    if params.num_partitions:
        P, radix = int(params.num_partitions), False
    else:
        P, radix = 1 << (params.radix_bits[0] + params.radix_bits[1]), True

    def segment_of(codes):
        u = np.ascontiguousarray(codes).view(np.uint64)
        q = (u & np.uint64(P - 1)) if radix else (u % np.uint64(P))
        if sub_bits:
            q = (q << np.uint64(sub_bits)) | ((u >> np.uint64(sub_shift)) & np.uint64((1 << sub_bits) - 1))
        return (q >> np.uint64(shift)).astype(np.int64)
    return nseg, segment_of


def codes_of(keys, params):
    kind = O.HASH_MURMUR3 if params.hash == phj.HASH_MURMUR3 else O.HASH_XXH3
    return O.hash_keys(kind, np.ascontiguousarray(keys, dtype=np.int64), params.hash_seed).view(np.int64)


def pack(R_shard, params, total_build, codes_elems, block_elems):
    """This rank's exchange block: its build codes grouped by segment, zero
    padded to codes_elems, then the num_segments + 1 uint32 bounds."""
    nseg, segment_of = geometry(params, total_build)
    codes = codes_of(R_shard[:, 0], params)
    seg = segment_of(codes)
    order = np.argsort(seg, kind="stable")
    block = np.zeros(block_elems, dtype=np.int64)
    block[:codes.shape[0]] = codes[order]
    bounds = np.zeros(nseg + 1, dtype=np.uint32)
    bounds[1:] = np.cumsum(np.bincount(seg, minlength=nseg))
    block[codes_elems:].view(np.uint32)[:nseg + 1] = bounds
    return block


def segments(recv, world, nseg, codes_elems, block_elems):
    """The gathered blocks as build segments (codes, bounds), as phj_group.h reads them."""
    segs = []
    for g in range(world):
        blk = recv[g * block_elems:(g + 1) * block_elems]
        b = blk[codes_elems:].view(np.uint32)[:nseg + 1].astype(np.int64)
        segs.append((blk[:b[nseg]], b))
    return segs


def same_block(a, b, nseg, codes_elems):
    """Bounds equal and every segment the same multiset of codes."""
    ba = a[codes_elems:].view(np.uint32)[:nseg + 1]
    bb = b[codes_elems:].view(np.uint32)[:nseg + 1]
    if not np.array_equal(ba, bb):
        return False
    for s in range(nseg):
        lo, hi = int(ba[s]), int(ba[s + 1])
        if not np.array_equal(np.sort(a[lo:hi]), np.sort(b[lo:hi])):
            return False
    return True
