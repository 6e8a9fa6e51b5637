"""Variant edit: CalculateRadiance's loop counters and flags (PState) as bit-fields of one register.
argv[1] = csrc dir."""
import os
import sys

p = os.path.join(sys.argv[1], "pt_program.h")
s = open(p).read()
old = """    int diffuseCount, hitType, bounce;
    bool coat, specular, sampleLight;
};"""
new = """    // the counters and flags packed into one register (bit-fields): diffuseCount <= 6, bounce <= 6,
    // hitType in [-100, 10]
    int diffuseCount : 4, hitType : 8, bounce : 4;
    bool coat : 1, specular : 1, sampleLight : 1;
};"""
assert old in s
s = s.replace(old, new, 1)
open(p, "w").write(s)
