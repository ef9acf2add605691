"""Test infrastructure: a pure-Python model of libstdc++ std::sort (introsort) over
PCL VoxelGrid's (key, index) pairs compared by key only, and of the row-D split of
that sort (fccf-pcr_amd/csrc/introsort.hip: plan_round, k_is_block; group.cpp):
the first r0 levels of segments longer than `tier` are run replicated, then the
children of level r0 - 1 are cut into rank ranges (bound j = the first child start
>= j * n / N) and each rank finishes only the segments starting in its range; the
rank-ordered concatenation of the ranges is the whole sort.  Small inputs only
(pure Python).  The oracle's std::sort (oracle_py.sort_pairs) is the reference.
"""
from __future__ import annotations

THRESHOLD = 16  # libstdc++ _S_threshold
INVALID = 0xFFFFFFFF


def _lg(n: int) -> int:
    return n.bit_length() - 1


def _median_to_first(a, result, x, y, z):
    k = lambda i: a[i][0]  # noqa: E731
    if k(x) < k(y):
        if k(y) < k(z):
            m = y
        elif k(x) < k(z):
            m = z
        else:
            m = x
    elif k(x) < k(z):
        m = x
    elif k(y) < k(z):
        m = z
    else:
        m = y
    a[result], a[m] = a[m], a[result]


def _unguarded_partition(a, first, last, pivot):
    p = a[pivot][0]
    while True:
        while a[first][0] < p:
            first += 1
        last -= 1
        while p < a[last][0]:
            last -= 1
        if not first < last:
            return first
        a[first], a[last] = a[last], a[first]
        first += 1


def _partition_pivot(a, first, last):
    mid = first + (last - first) // 2
    _median_to_first(a, first, first + 1, mid, last - 1)
    return _unguarded_partition(a, first + 1, last, first)


def _adjust_heap(a, base, hole, length, value):
    top = hole
    child = hole
    while child < (length - 1) // 2:
        child = 2 * (child + 1)
        if a[base + child][0] < a[base + child - 1][0]:
            child -= 1
        a[base + hole] = a[base + child]
        hole = child
    if (length & 1) == 0 and child == (length - 2) // 2:
        child = 2 * (child + 1)
        a[base + hole] = a[base + child - 1]
        hole = child - 1
    parent = (hole - 1) // 2
    while hole > top and a[base + parent][0] < value[0]:
        a[base + hole] = a[base + parent]
        hole = parent
        parent = (hole - 1) // 2
    a[base + hole] = value


def _heap_sort(a, first, last):
    n = last - first
    if n < 2:
        return
    for parent in range((n - 2) // 2, -1, -1):
        _adjust_heap(a, first, parent, n, a[first + parent])
    for end in range(n - 1, 0, -1):
        v = a[first + end]
        a[first + end] = a[first]
        _adjust_heap(a, first, 0, end, v)


def _introsort_loop(a, first, last, depth):
    while last - first > THRESHOLD:
        if depth == 0:
            _heap_sort(a, first, last)
            return
        depth -= 1
        cut = _partition_pivot(a, first, last)
        _introsort_loop(a, cut, last, depth)
        last = cut


def _insertion_sort(a, first, last):
    """Stable insertion sort of [first, last) by key (the final insertion sort, which
    leaves each leaf segment stably sorted)."""
    for i in range(first + 1, last):
        v = a[i]
        j = i
        while j > first and v[0] < a[j - 1][0]:
            a[j] = a[j - 1]
            j -= 1
        a[j] = v


def pairs_of(keys):
    return [(int(k), i) for i, k in enumerate(keys) if int(k) != INVALID]


def std_sort(keys) -> list[int]:
    """The input positions of the valid keys in std::sort order."""
    a = pairs_of(keys)
    n = len(a)
    if n > 1:
        _introsort_loop(a, 0, n, 2 * _lg(n))
        _insertion_sort(a, 0, n)
    return [i for _, i in a]


def rank_bounds(child_starts, n, world):
    """plan_round's rule: bound j = the first child start >= j * n / world."""
    b = [0] + [n] * world
    for j in range(1, world):
        c = [f for f in child_starts if f * world >= j * n]
        b[j] = min(c) if c else n
    return b


def sharded_rank(keys, rank: int, world: int, tier: int, r0: int):
    """Rank `rank`'s part of the row-D sort: ((lo, hi), the input positions at sorted
    positions lo..hi-1).  Levels < r0 run every segment longer than `tier` (all ranks
    alike); segments of <= tier elements are owned and finished at once by the rank
    whose range holds their start; from level r0 on only this rank's segments."""
    a = pairs_of(keys)
    n = len(a)
    if n <= 1:
        return (0, n), [i for _, i in a]
    owned = []  # (f, l, depth) finished later by their range's rank
    level = [(0, n, 2 * _lg(n))]
    children = []
    for _ in range(r0):
        children = []
        nxt = []
        for f, l, d in level:
            if l - f > tier and d > 0:
                c = _partition_pivot(a, f, l)
                children += [(f, c, d - 1), (c, l, d - 1)]
            else:
                owned.append((f, l, d))
        for f, l, d in children:
            if l - f > tier and d > 0:
                nxt.append((f, l, d))
            else:
                owned.append((f, l, d))
        level = nxt
        if not level:
            break
    b = rank_bounds([f for f, _, _ in children], n, world) if children else [0] + [n] * world
    lo, hi = b[rank], b[rank + 1]
    for f, l, d in level + owned:
        if lo <= f < hi:
            _introsort_loop(a, f, l, d)
    _insertion_sort(a, lo, hi)
    return (lo, hi), [i for _, i in a[lo:hi]]
