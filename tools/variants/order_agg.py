"""Variant edit: pt_order_build's LDS bucket atomics aggregated per wave (one atomic per distinct
bucket among the wave's 64 tiles, ranks by popcount), instead of one per tile. argv[1] = csrc dir."""
import os
import sys

p = os.path.join(sys.argv[1], "pt_kernels.hip")
s = open(p).read()
helper = """// one LDS atomic per distinct bucket among the wave's lanes (all lanes active): returns this lane's
// slot, cnt[b] before the wave's adds + its rank among the lanes with the same bucket
PT_D unsigned waveAdd(unsigned* cnt, unsigned b, bool valid)
{
    const int lane = __lane_id();
    const unsigned long long below = (1ull << lane) - 1ull;
    unsigned long long todo = __ballot(valid);
    unsigned pos = 0u;
    while (todo) {
        const int leader = __builtin_ctzll(todo);
        const unsigned bl = (unsigned)__shfl((int)b, leader, 64);
        const unsigned long long m = todo & __ballot(b == bl);
        unsigned base = 0u;
        if (lane == leader) base = atomicAdd(&cnt[bl], (unsigned)__popcll(m));
        base = (unsigned)__shfl((int)base, leader, 64);
        if ((m >> lane) & 1ull) pos = base + (unsigned)__popcll(m & below);
        todo &= ~m;
    }
    return pos;
}

"""
anchor = "// Builds order[] (a permutation of the ntiles 16x16 tiles)"
assert anchor in s
s = s.replace(anchor, helper + anchor, 1)
old1 = "                if (t < ntiles) atomicAdd(&cnt[b], 1u);\n"
assert old1 in s
s = s.replace(old1, "                waveAdd(cnt, b, t < ntiles);\n", 1)
old2 = """            if (t < ntiles) {
                const unsigned pos = atomicAdd(&cnt[(bk[j >> 2] >> (8 * (j & 3))) & 255u], 1u);
                if (pos < ntiles) order[pos] = t;
            }"""
assert old2 in s
s = s.replace(old2, """            const unsigned pos = waveAdd(cnt, (bk[j >> 2] >> (8 * (j & 3))) & 255u, t < ntiles);
            if (t < ntiles && pos < ntiles) order[pos] = t;""", 1)
open(p, "w").write(s)
