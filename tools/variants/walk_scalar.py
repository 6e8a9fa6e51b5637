"""Variant edit: the child-pair walk reads a record through the scalar cache when every active lane of
the wave is at that record (ballot == exec), instead of four vector loads. argv[1] = csrc dir.
argv[2] (optional) = 'notex': only in the variants without PBR maps."""
import os
import sys

d = sys.argv[1]
only_notex = len(sys.argv) > 2 and sys.argv[2] == "notex"
p = os.path.join(d, "pt_device.h")
s = open(p).read()
old_t = "typedef unsigned int vu2 __attribute__((ext_vector_type(2)));\n"
s = s.replace(old_t, old_t + "typedef unsigned int vu8 __attribute__((ext_vector_type(8)));\n#define PT_CONST_AS __attribute__((address_space(4)))\n", 1)
old = """        const uint32_t off = code & ~kLeafBit;
        const float4 r0 = ldRec4(b.rec, off), r1 = ldRec4(b.rec, off + 16u), r2 = ldRec4(b.rec, off + 32u);
        const float2 r3 = ldRec2(b.rec, off + 48u);
"""
new = """        const uint32_t off = code & ~kLeafBit;
        float4 r0, r1, r2;
        float2 r3;
        if (SCALAR_COND __builtin_amdgcn_ballot_w64(off == __builtin_amdgcn_readfirstlane(off)) == __builtin_amdgcn_read_exec()) {
            const uint32_t so = __builtin_amdgcn_readfirstlane(off);
            const PT_CONST_AS char* sbase = (const PT_CONST_AS char*)a.bvh_pairs;
            const vu8 v = *(const PT_CONST_AS vu8*)(sbase + so);
            const vu4 w = *(const PT_CONST_AS vu4*)(sbase + so + 32u);
            r0 = make_float4(__uint_as_float(v.s0), __uint_as_float(v.s1), __uint_as_float(v.s2), __uint_as_float(v.s3));
            r1 = make_float4(__uint_as_float(v.s4), __uint_as_float(v.s5), __uint_as_float(v.s6), __uint_as_float(v.s7));
            r2 = make_float4(__uint_as_float(w.x), __uint_as_float(w.y), __uint_as_float(w.z), __uint_as_float(w.w));
            r3 = make_float2(0.0f, 0.0f);
            if (!(__builtin_amdgcn_readfirstlane(code) & kLeafBit)) {
                const vu2 c = *(const PT_CONST_AS vu2*)(sbase + so + 48u);
                r3 = make_float2(__uint_as_float(c.x), __uint_as_float(c.y));
            }
        } else {
            r0 = ldRec4(b.rec, off); r1 = ldRec4(b.rec, off + 16u); r2 = ldRec4(b.rec, off + 32u);
            r3 = ldRec2(b.rec, off + 48u);
        }
""".replace("SCALAR_COND", "kScalarWalk &&" if only_notex else "")
assert old in s
s = s.replace(old, new, 1)
if only_notex:
    # bvhWalkPairs is not templated on the program: pass the choice as a template parameter
    s = s.replace("template <class Stk>\nPT_D void bvhWalkPairs(", "template <bool kScalarWalk = false, class Stk>\nPT_D void bvhWalkPairs(", 1)
    t = os.path.join(d, "pt_trace.h")
    ts = open(t).read()
    o2 = "else bvhWalkPairs(a, O, D, inv, dbl, rootT, h.t, st, br, anyHit);"
    assert o2 in ts
    ts = ts.replace(o2, "else bvhWalkPairs<!kHasTex<PROG>>(a, O, D, inv, dbl, rootT, h.t, st, br, anyHit);")
    open(t, "w").write(ts)
open(p, "w").write(s)
