"""CPU models of the r4 per-row Lomuto forms (the algorithms the gfx950
kernels implement; the kernels themselves are checked bit-exact on the GPU by
tests/test_gpu_parity.py's buildKDTree and rows tests):

* the block pass with one barrier per chunk (navgpu.hip block_nth_element):
  per chunk the waves publish their small / large ballots and elements, then
  each lane follows its tape chain through them (tape_jump per run of
  smalls, earlier chunks' final tape, published elements);
* the register-resident nth_element for windows of at most 64 positions
  (wave_nth_element_regs): ballots, shuffle-resolved tape, two forward
  permutes per pass.

Both must reproduce the reference nth_element (utils/kdtree.c:20-52: Lomuto,
pivot = last, `<= 0` goes left) exactly, on random, sorted, reversed and
duplicate-heavy windows."""
import numpy as np
import pytest

W = 64


def tape_jump(p, sp, lbelow, wave_p0):
    """navgpu.hip tape_jump: the first position below p's run of smalls
    that p's tape chain reaches (L = p - sp larges before p)."""
    k = p - sp
    s = (wave_p0 + lbelow.bit_length()) if lbelow else wave_p0
    return p - k * ((p - s + k) // k)


def lomuto_pass(key, P, first, last):
    pe = P[last]
    pk = key[pe]
    i = first
    for j in range(first, last):
        if key[P[j]] - pk <= 0.0:
            P[j], P[i] = P[i], P[j]
            i += 1
    P[last] = P[i]
    P[i] = pe
    return i


def lomuto_nth(key, P, first, last, nth):
    while first < last:
        i = lomuto_pass(key, P, first, last)
        if i == nth:
            return
        if i < nth:
            first = i + 1
        else:
            last = i - 1


def block_pass(key, P, first, last, bd):
    """One Lomuto pass as block_nth_element (r4) runs it: chunks of bd
    positions, bd / 64 waves, one barrier per chunk."""
    pe = P[last]
    pk = key[pe]
    m = last - first
    T = {}
    S = 0
    nw = bd // W
    for cs in range(0, m, bd):
        E, small, large = {}, {}, {}
        for t in range(bd):
            p = cs + t
            act = p < m
            e = P[first + p] if act else 0
            E[t] = e
            small[t] = act and key[e] - pk <= 0.0
            large[t] = act and not small[t]
        SB = [sum(1 << l for l in range(W) if small[w * W + l]) for w in range(nw)]
        LB = [sum(1 << l for l in range(W) if large[w * W + l]) for w in range(nw)]
        before = [sum(bin(SB[x]).count("1") for x in range(w)) for w in range(nw)]
        out_t, out_p = {}, {}
        for t in range(bd):
            p = cs + t
            if p >= m:
                continue
            w, l = divmod(t, W)
            sp = S + before[w] + bin(SB[w] & ((1 << l) - 1)).count("1")
            if large[t] or sp == p:
                val = E[t]
            else:
                y = tape_jump(p, sp, LB[w] & ((1 << l) - 1), cs + w * W)
                while True:
                    if y < cs:
                        val = T[first + y]
                        break
                    wy, ly = divmod(y - cs, W)
                    spy = S + before[wy] + bin(SB[wy] & ((1 << ly) - 1)).count("1")
                    if (LB[wy] >> ly) & 1 or spy == y:
                        val = E[y - cs]
                        break
                    y = tape_jump(y, spy, LB[wy] & ((1 << ly) - 1), cs + wy * W)
            out_t[first + p] = val
            if small[t]:
                out_p[first + sp] = E[t]
        T.update(out_t)
        for k, v in out_p.items():
            P[k] = v
        S += sum(bin(x).count("1") for x in SB)
    for q in range(S, m):
        P[last if q == S else first + q] = T[first + q]
    P[first + S] = pe
    return first + S


def regs_nth(key, P, first, last, nth):
    """wave_nth_element_regs: the window in lanes, permutes per pass."""
    n = last - first + 1
    e = [P[first + l] if l < n else 0 for l in range(W)]
    a, b, nl = 0, n - 1, nth - first
    while a < b:
        pe = e[b]
        pk = key[pe]
        small = [a <= l < b and key[e[l]] - pk <= 0.0 for l in range(W)]
        large = [a <= l < b and not small[l] for l in range(W)]
        bal = sum(1 << l for l in range(W) if small[l])
        lbal = sum(1 << l for l in range(W) if large[l])
        ps = a + bin(bal).count("1")
        sp = [a + bin(bal & ((1 << l) - 1)).count("1") for l in range(W)]
        w = [("p", tape_jump(l, sp[l], lbal & ((1 << l) - 1), 0)) if small[l] and sp[l] != l
             else ("r", e[l]) for l in range(W)]
        while any(x[0] == "p" for x in w):
            w = [w[x[1]] if x[0] == "p" else x for x in w]
        v1, v2 = {}, {}
        for l in range(W):
            if small[l]:
                v1[sp[l]] = e[l]
            if ps <= l < b:
                v2[b if l == ps else l] = w[l][1]
        e = [v1[l] if a <= l < ps else pe if l == ps else v2[l] if ps < l <= b else e[l]
             for l in range(W)]
        if ps == nl:
            break
        if ps < nl:
            a = ps + 1
        else:
            b = ps - 1
    for l in range(n):
        P[first + l] = e[l]


def _keys(rng, kind, n):
    if kind == "random":
        return list(rng.uniform(0, 1, n))
    if kind == "sorted":
        return list(np.sort(rng.uniform(0, 1, n)))
    if kind == "reversed":
        return list(np.sort(rng.uniform(0, 1, n))[::-1])
    return list(np.round(rng.uniform(0, 4, n)))  # duplicates


@pytest.mark.parametrize("kind", ["random", "sorted", "reversed", "duplicates"])
def test_block_pass_equals_lomuto(kind):
    rng = np.random.default_rng(len(kind))
    for trial in range(12):
        first = int(rng.integers(0, 64))
        n = int(rng.integers(first + 300, 1400))
        key = _keys(rng, kind, n)
        P0 = list(rng.permutation(n))
        last = int(rng.integers(first + 256, n))
        a, b = P0.copy(), P0.copy()
        ia = lomuto_pass(key, a, first, last)
        ib = block_pass(key, b, first, last, 512 if trial % 2 else 1024)
        assert ia == ib and a == b, (kind, trial)


@pytest.mark.parametrize("kind", ["random", "sorted", "reversed", "duplicates"])
def test_register_nth_equals_lomuto(kind):
    rng = np.random.default_rng(10 + len(kind))
    for trial in range(150):
        n = int(rng.integers(2, 65))
        key = _keys(rng, kind, n)
        P0 = list(rng.permutation(n))
        nth = int(rng.integers(0, n))
        a, b = P0.copy(), P0.copy()
        lomuto_nth(key, a, 0, n - 1, nth)
        regs_nth(key, b, 0, n - 1, nth)
        assert a == b, (kind, trial, n, nth)
