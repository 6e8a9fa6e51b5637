#!/usr/bin/env python3
"""oracle/xcheck/transcribe.py — TEST INFRASTRUCTURE (build container only; needs /root/reference).

Mechanical GLSL -> C++ transcription of the reference's path-tracing fragment shaders, to check
the C oracle's hand restatement of them. The GLSL text is taken as it stands
in the reference's JS files (the BABYLON.Effect.ShadersStore / IncludesShadersStore template
literals of js/PathTracingCommon.js and js/<Scene>_FragmentShader.js), its #include<...> chunks
are expanded, and a fixed set of purely syntactic rewrites turns it into C++20 over
oracle/xcheck/glsl_shim.h:

  * float literals get an `f` suffix (GLSL float literals are single precision);
  * `#version` / `precision` lines go; every `#define` is preceded by an `#undef`;
  * 2-4 letter swizzles `.xzy` -> `.sw<0,2,1>()` (1-letter ones are union members);
  * constructor calls `vec3(...)`, `Quad(...)` -> `vec3{...}`, `Quad{...}` (braces also fix the
    left-to-right evaluation order of the arguments, which rng() calls depend on);
  * globals become thread_local (one copy per fragment invocation) except uniforms; arrays become
    bounds-safe glx::garr; local declarations without an initialiser are zero-initialised (the
    pinned meaning of an unwritten GLSL variable);
  * `out` / `inout` parameters become references with a local copy written back on return;
  * main() becomes xc_main().

Nothing is interpreted: no expression is re-associated, reordered or simplified. The generated
C++ goes to oracle/_ref/ only (never into git): it is the reference's source in another syntax.
Statements that hold more than one rng() / blueNoise_rand() call outside a constructor's
braces are reported (C++ leaves their order unspecified) so that a human checks them.

usage: transcribe.py PROGRAM OUT.cpp   with PROGRAM one of: cornell gltf hdri sky quadric screen_output screen_copy
"""
import os
import re
import sys

REF = os.environ.get("PT_REFERENCE", "/root/reference")
SCENES = {   # program -> (file, ShadersStore key)
    "cornell": ("BabylonPathTracing_FragmentShader.js", "pathTracingFragmentShader"),
    "gltf": ("GLTFModelPathTracing_FragmentShader.js", "pathTracingFragmentShader"),
    "hdri": ("HDRIEnvironmentPathTracing_FragmentShader.js", "pathTracingFragmentShader"),
    "sky": ("PhysicalSkyModel_FragmentShader.js", "pathTracingFragmentShader"),
    "quadric": ("TransformedQuadricGeometry_FragmentShader.js", "pathTracingFragmentShader"),
    "screen_output": ("PathTracingCommon.js", "screenOutputFragmentShader"),
    "screen_copy": ("PathTracingCommon.js", "screenCopyFragmentShader"),
}
VEC_TYPES = ["vec2", "vec3", "vec4", "ivec2", "ivec3", "ivec4", "uvec2", "uvec3", "uvec4", "mat3", "mat4"]
SCALARS = ["float", "int", "uint", "bool"]
SWZ_SETS = ["xyzw", "rgba", "stpq"]


def shader_store(path):
    text = open(path).read()
    pat = re.compile(r"BABYLON\.Effect\.(?:ShadersStore|IncludesShadersStore)\s*\[\s*['\"](\w+)['\"]\s*\]\s*=\s*`(.*?)`", re.S)
    return {m.group(1): m.group(2) for m in pat.finditer(text)}


def expand(text, chunks, depth=0):
    if depth > 8:
        raise RuntimeError("include depth")
    return re.sub(r"#include\s*<\s*(\w+)\s*>", lambda m: expand(chunks[m.group(1)], chunks, depth + 1), text)


def strip_comments(text):
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    return re.sub(r"//[^\n]*", "", text)


def float_literals(text):
    num = re.compile(r"(?<![\w.])((?:\d+\.\d*|\.\d+)(?:[eE][+-]?\d+)?|\d+[eE][+-]?\d+)(?![\w.])")
    return num.sub(lambda m: m.group(1) + "f", text)


def swizzles(text):
    def rep(m):
        s = m.group(1)
        for st in SWZ_SETS:
            if all(c in st for c in s):
                return ".sw<%s>()" % ",".join(str(st.index(c)) for c in s)
        return m.group(0)
    return re.sub(r"(?<=[\w\)\]])\.([xyzwrgbastpq]{2,4})\b(?!\s*\()", rep, text)


def braces_for_constructors(text, ctor_names):
    """vec3( ... ) -> vec3{ ... } for every constructor call, nesting-aware."""
    out, stack = [], []
    ident = re.compile(r"([A-Za-z_]\w*)\s*$")
    for ch in text:
        if ch == "(":
            m = ident.search("".join(out[-64:]))
            is_ctor = bool(m) and m.group(1) in ctor_names
            stack.append(is_ctor)
            out.append("{" if is_ctor else "(")
        elif ch == ")":
            out.append("}" if (stack.pop() if stack else False) else ")")
        else:
            out.append(ch)
    return "".join(out)


def split_top(text):
    """Top-level items: ('pp', line) | ('struct', text) | ('func', text) | ('decl', text)."""
    items, i, n = [], 0, len(text)
    while i < n:
        if text[i].isspace():
            i += 1
            continue
        if text[i] == "#":
            j = text.find("\n", i)
            j = n if j < 0 else j
            items.append(("pp", text[i:j]))
            i = j
            continue
        # scan to the end of the item: a ';' at depth 0, or a '}' closing a depth-0 '{' (functions)
        j, depth, kind = i, 0, None
        while j < n:
            c = text[j]
            if c == "{":
                depth += 1
            elif c == "}":
                depth -= 1
                if depth == 0:
                    rest = text[j + 1:].lstrip()
                    if text[i:].startswith("struct"):
                        k = text.index(";", j)
                        items.append(("struct", text[i:k + 1]))
                        j = k + 1
                    else:
                        items.append(("func", text[i:j + 1]))
                        j += 1
                    kind = "done"
                    break
            elif c == ";" and depth == 0:
                items.append(("decl", text[i:j + 1]))
                j += 1
                kind = "done"
                break
            j += 1
        if kind is None:
            raise RuntimeError("unterminated top-level item: %r" % text[i:i + 80])
        i = j
    return items


def split_commas(s):
    parts, depth, cur = [], 0, []
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
    parts.append("".join(cur))
    return [p.strip() for p in parts if p.strip()]


def array_decl(decl_type, declarator):
    m = re.match(r"(\w+)\s*\[\s*([^\]]+)\]\s*$", declarator)
    if m:
        return "glx::garr<%s, %s> %s" % (decl_type, m.group(2), m.group(1))
    return None


def transcribe(scene):
    common = shader_store(os.path.join(REF, "js", "PathTracingCommon.js"))
    fname, key = SCENES[scene]
    scene_store = shader_store(os.path.join(REF, "js", fname))
    src = expand(scene_store[key], common)
    src = strip_comments(src)
    src = "\n".join(l for l in src.split("\n") if not re.match(r"\s*(#version|precision)\b", l))
    structs = re.findall(r"\bstruct\s+(\w+)", src)
    types = VEC_TYPES + SCALARS + structs + ["sampler2D"]
    src = float_literals(src)
    src = swizzles(src)
    ctors = set(VEC_TYPES + structs)

    uniforms, globals_, out = [], [], []
    type_re = "|".join(types)
    for kind, text in split_top(src):
        if kind in ("decl", "func"):
            text = braces_for_constructors(text, ctors)
        if kind == "pp":
            m = re.match(r"#define\s+(\w+)", text)
            if m:
                out.append("#undef %s" % m.group(1))
            out.append(text)
        elif kind == "struct":
            out.append(text)
        elif kind == "decl":
            m = re.match(r"(uniform|out|in|const)?\s*(%s)\s+(.*);$" % type_re, text.strip(), re.S)
            if not m:
                raise RuntimeError("unhandled top-level declaration: %r" % text)
            qual, ty, decls = m.group(1), m.group(2), split_commas(m.group(3))
            if any("(" in d for d in decls):
                raise RuntimeError("function prototype not handled: %r" % text)
            if qual not in ("uniform", "const") and any("=" in d for d in decls):
                raise RuntimeError("initialised global not handled (per-invocation reset): %r" % text)
            if qual == "uniform":
                for d in decls:
                    uniforms.append((ty, d))
                out.append("%s %s;" % (ty, ", ".join(decls)))
                continue
            parts = []
            for d in decls:
                a = array_decl(ty, d)
                if a:
                    out.append("thread_local %s;" % a)
                    globals_.append(d.split("[")[0].strip())
                else:
                    parts.append(d)
                    globals_.append(d.split("=")[0].strip())
            if parts:
                out.append("%s%s %s;" % ("" if qual == "const" else "thread_local ", ty, ", ".join(parts)))
        else:
            out.append(function(text, type_re))
    return "\n".join(out), uniforms, globals_


def function(text, type_re):
    head, body = text[:text.index("{")], text[text.index("{"):]
    m = re.match(r"\s*(\w+)\s+(\w+)\s*\((.*)\)\s*$", head, re.S)
    if not m:
        raise RuntimeError("unhandled function head: %r" % head)
    ret, name, params = m.groups()
    if name == "main":
        name = "xc_main"
    plist, prologue = [], []
    for p in split_commas(params):
        toks = p.split()
        if toks == ["void"]:
            continue
        quals = [t for t in toks[:-2] if t in ("const", "in", "out", "inout", "highp", "mediump", "lowp")]
        ty, pname = toks[-2], toks[-1]
        if "out" in quals or "inout" in quals:
            ref = pname + ("__out" if "out" in quals else "__inout")
            plist.append("%s& %s" % (ty, ref))
            init = "{}" if "out" in quals else " = %s" % ref
            prologue.append("%s %s%s; glx::OutCopy<%s> %s__cp{%s, %s};" % (ty, pname, init, ty, pname, ref, pname))
        else:
            plist.append("%s %s" % (ty, pname))
    body = zero_init_locals(body, type_re)
    body = "{ " + " ".join(prologue) + body[1:]
    return "%s %s(%s)\n%s" % (ret, name, ", ".join(plist), body)


def zero_init_locals(body, type_re):
    pat = re.compile(r"(?<=[;{}])(\s*)(const\s+)?(%s)(\s+)([^;(){}]*);" % type_re)

    def rep(m):
        decls = split_commas(m.group(5))
        fixed = [d if ("=" in d or "[" in d) else d + "{}" for d in decls]
        if any("[" in d and "=" not in d for d in decls):
            fixed = [d + "{}" if ("[" in d and "=" not in d) else f for d, f in zip(decls, fixed)]
        return "%s%s%s%s%s;" % (m.group(1), m.group(2) or "", m.group(3), m.group(4), ", ".join(fixed))
    return pat.sub(rep, body)


def order_report(code):
    """Statements with two or more rng()/blueNoise_rand() calls outside constructor braces."""
    flagged = []
    for stmt in re.split(r"[;{}]", code):
        if len(re.findall(r"\b(rng|blueNoise_rand)\s*\(", stmt)) >= 2:
            flagged.append(" ".join(stmt.split()))
    return flagged


SETTER = {
    "float": "xc_u = xc_v[0];",
    "int": "xc_u = (int)xc_v[0];",
    "bool": "xc_u = xc_v[0] != 0.0f;",
    "vec2": "xc_u = vec2(xc_v[0], xc_v[1]);",
    "vec3": "xc_u = vec3(xc_v[0], xc_v[1], xc_v[2]);",
    "vec4": "xc_u = vec4(xc_v[0], xc_v[1], xc_v[2], xc_v[3]);",
    "mat4": "for (int xc_c = 0; xc_c < 4; xc_c++) for (int xc_r = 0; xc_r < 4; xc_r++) xc_u.c[xc_c].v[xc_r] = xc_v[4 * xc_c + xc_r];",
}
NEEDS = {"float": 1, "int": 1, "bool": 1, "vec2": 2, "vec3": 3, "vec4": 4, "mat4": 16}


def generate(scene, out_path):
    code, uniforms, globals_ = transcribe(scene)
    lines = ["// GENERATED by oracle/xcheck/transcribe.py from /root/reference/js/%s (%s) and js/PathTracingCommon.js" % SCENES[scene],
             "// (build-container artefact under oracle/_ref/: never committed)",
             '#include "glsl_shim.h"', '#include "harness.inc"', "namespace glx {", code]
    lines.append("vec4 xc_frag_color() { return glFragColor; }")
    lines.append("void xc_reset_globals() {")
    for g in globals_:
        lines.append("    std::memset((void*)&%s, 0, sizeof(%s));" % (g, g))
    lines.append("}")
    lines.append("}  // namespace glx")
    lines.append('extern "C" int xc_set_uniform(const char* xc_name, const float* xc_v, int xc_n) {')
    lines.append("    using namespace glx;")
    for ty, name in uniforms:
        if ty == "sampler2D":
            continue
        if ty not in SETTER:
            raise RuntimeError("uniform type %s" % ty)
        lines.append('    if (!std::strcmp(xc_name, "%s")) { if (xc_n < %d) return -2; auto& xc_u = %s; %s return 0; }'
                     % (name, NEEDS[ty], name, SETTER[ty]))
    lines.append("    return 1;   // not a uniform of this program (ignored, as Babylon ignores it)")
    lines.append("}")
    lines.append('extern "C" int xc_set_sampler(const char* xc_name, const void* xc_data, int xc_w, int xc_h, int xc_f32) {')
    lines.append("    using namespace glx;")
    for ty, name in uniforms:
        if ty == "sampler2D":
            lines.append('    if (!std::strcmp(xc_name, "%s")) { %s.data = xc_data; %s.w = xc_w; %s.h = xc_h; %s.f32 = xc_f32; return 0; }'
                         % (name, name, name, name, name))
    lines.append("    return 1;")
    lines.append("}")
    with open(out_path, "w") as f:
        f.write("\n".join(lines) + "\n")
    return order_report(code)


if __name__ == "__main__":
    flagged = generate(sys.argv[1], sys.argv[2])
    for s in flagged:
        print("ORDER-CHECK:", s)
