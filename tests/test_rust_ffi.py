"""The Rust drop-in binding (rust/src/rtm_ffi.rs) against include/rtm.h.

Rust is not installed in this image, so rustc cannot check the binding; this CPU
test does instead.  It parses the header (constants, structs, every function
prototype) and the binding (consts, #[repr(C)] structs, the extern "C" block) and
requires: the same function set, each with the same argument count, argument C
types and return type (mapped to their Rust equivalents); the same structs with
the same fields in the same order and types; the same constants; and struct
layouts (size, field offsets computed with C rules) equal to abi.py's ctypes
mirror, which tests/test_abi.py pins to the C compiler's view of the header.  Any
change to rtm.h without the binding fails here."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rtm.h")
RUST = os.path.join(ROOT, "rust", "src", "rtm_ffi.rs")

C_BASE = {"int": "i32", "int32_t": "i32", "int64_t": "i64", "uint8_t": "u8", "float": "f32", "double": "f64",
          "char": "c_char", "void": "c_void"}
RUST_KEYWORDS = {"type": "type_"}


def _strip_c(src):
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return re.sub(r"//[^\n]*", "", src)


def c_constants(src):
    return {m.group(1): int(m.group(2), 0) for m in re.finditer(r"#define\s+(RTM_\w+)\s+(-?(?:0x[0-9a-fA-F]+|\d+))\b",
                                                              src)}


def c_type_to_rust(tokens, array=False, is_return=False):
    """Rust spelling of a C type given as tokens (no declarator name): the base is
    const iff 'const' precedes the first '*'; a 'const' after a '*' makes that
    pointer itself const, i.e. the next level's pointee.  An array parameter decays
    to a pointer."""
    if array:
        tokens = tokens + ["*"]
    base, base_const, levels = None, False, []  # levels: constness of each pointer, innermost first
    for t in tokens:
        if t == "const":
            if levels:
                levels[-1] = True
            else:
                base_const = True
        elif t == "*":
            levels.append(False)
        else:
            assert base is None, tokens
            base = t
    if not levels:
        return "()" if (base == "void" and is_return) else C_BASE.get(base, base)
    s = C_BASE.get(base, base)
    pointee_const = base_const
    for const_ptr in levels:
        s = ("*const " if pointee_const else "*mut ") + s
        pointee_const = const_ptr
    return s


def _tok(s):
    return re.findall(r"\w+|\*", s)


def c_functions(src):
    src = _strip_c(src)
    out = {}
    for m in re.finditer(r"^\s*([\w\s\*]+?)\b(rtm_\w+)\s*\(([^;{]*?)\)\s*;", src, flags=re.M):
        ret, name, args = m.group(1), m.group(2), m.group(3)
        if ret.strip().startswith("typedef"):
            continue
        rs = c_type_to_rust(_tok(ret), is_return=True)
        params = []
        if args.strip() not in ("", "void"):
            for a in args.split(","):
                a = a.strip()
                arr = re.search(r"\[\s*\w*\s*\]\s*$", a)
                a = re.sub(r"\[\s*\w*\s*\]\s*$", "", a)
                toks = _tok(a)
                params.append((toks[-1], c_type_to_rust(toks[:-1], array=bool(arr))))
        out[name] = (params, rs)
    return out


def c_structs(src, consts):
    src = _strip_c(src)
    out = {}
    for m in re.finditer(r"typedef\s+struct\s+(\w+)\s*\{(.*?)\}\s*(\w+)\s*;", src, flags=re.S):
        name, body = m.group(1), m.group(2)
        fields = []
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            m2 = re.match(r"((?:const\s+)?\w+\s*\**)\s*(.*)$", decl, flags=re.S)
            base_toks = _tok(m2.group(1))
            for d in m2.group(2).split(","):
                d = d.strip()
                stars = d.count("*")
                d = d.replace("*", "").strip()
                arr = re.match(r"(\w+)\s*\[\s*(\w+)\s*\]", d)
                fname = arr.group(1) if arr else d
                t = c_type_to_rust(base_toks + ["*"] * stars)
                if arr:
                    n = arr.group(2)
                    t = f"[{t}; {consts.get(n, n)}]"
                fields.append((RUST_KEYWORDS.get(fname, fname), t))
        out[name] = fields
    return out


def _norm(t):
    t = re.sub(r"\s+", " ", t.strip())
    t = re.sub(r"\*\s*(const|mut)\s+", r"*\1 ", t)
    return re.sub(r"\[\s*(.*?)\s*;\s*(.*?)\s*\]", r"[\1; \2]", t)


def rust_items(src):
    body = re.sub(r"//[^\n]*", "", src)
    consts = {m.group(1): int(m.group(2), 0) for m in re.finditer(r"pub const (RTM_\w+)\s*:\s*i32\s*=\s*(-?(?:0x[0-9a-fA-F]+|\d+))\s*;",
                                                              body)}
    structs = {}
    for m in re.finditer(r"#\[repr\(C\)\]\s*(?:#\[derive\([^\]]*\)\]\s*)?pub struct (\w+)\s*\{(.*?)\}", body, flags=re.S):
        fields = re.findall(r"\bpub (\w+)\s*:\s*([^,]+?)\s*,", m.group(2))
        structs[m.group(1)] = [(n, _norm(t)) for n, t in fields]
    ext = re.search(r'extern "C"\s*\{(.*)\n\}', body, flags=re.S).group(1)
    fns = {}
    for m in re.finditer(r"pub fn (\w+)\s*\((.*?)\)\s*(?:->\s*([^;]+?))?\s*;", ext, flags=re.S):
        params = []
        args = m.group(2).strip()
        if args:
            for a in args.split(","):
                if a.strip():
                    n, t = a.split(":", 1)
                    params.append((n.strip(), _norm(t)))
        fns[m.group(1)] = (params, _norm(m.group(3)) if m.group(3) else "()")
    return consts, structs, fns


@pytest.fixture(scope="module")
def parsed():
    hsrc = open(HEADER).read()
    consts = c_constants(hsrc)
    return dict(c_consts=consts, c_fns=c_functions(hsrc), c_structs=c_structs(hsrc, consts),
                rust=rust_items(open(RUST).read()))


def test_every_header_function_is_bound_with_its_c_types(parsed):
    c_fns, (_, _, r_fns) = parsed["c_fns"], parsed["rust"]
    # every rtm_* name the header declares (tests/test_abi.py's scan) was parsed as a prototype
    src = _strip_c(open(HEADER).read())
    assert set(c_fns) == set(re.findall(r"\b(rtm_[a-z0-9_]+)\s*\(", src))
    assert set(r_fns) == set(c_fns), (sorted(set(c_fns) - set(r_fns)), sorted(set(r_fns) - set(c_fns)))
    for name, (cparams, cret) in c_fns.items():
        rparams, rret = r_fns[name]
        assert len(rparams) == len(cparams), (name, rparams, cparams)
        for (cn, ct), (rn, rt) in zip(cparams, rparams):
            assert rt == _norm(ct), (name, cn, ct, rn, rt)
        assert rret == _norm(cret), (name, cret, rret)


def test_headline_and_multi_gpu_calls_are_bound(parsed):
    _, _, r_fns = parsed["rust"]
    for n in ("rtm_render_frames_async", "rtm_ctx_set_lanes", "rtm_ctx_set_batch", "rtm_render_multi",
              "rtm_group_create_rank", "rtm_group_synchronize", "rtm_ctx_alloc", "rtm_ctx_copy_to_host"):
        assert n in r_fns, n
    params, _ = r_fns["rtm_render_frames_async"]
    assert params[-1] == ("out_rgba_dev", "*const *mut f32")  # float* const* out_rgba_dev


def test_structs_match_header_fields(parsed):
    c_st, (_, r_st, _) = parsed["c_structs"], parsed["rust"]
    assert set(c_st) <= set(r_st)
    for name, fields in c_st.items():
        assert r_st[name] == [(n, _norm(t)) for n, t in fields], name
    # the opaque handles
    for name in ("rtm_ctx", "rtm_group", "rtm_viewport"):
        assert r_st[name] == [], name


def test_constants_match_header(parsed):
    r_consts = parsed["rust"][0]
    assert r_consts == parsed["c_consts"]


_SIZES = {"i32": (4, 4), "i64": (8, 8), "f64": (8, 8), "f32": (4, 4), "u8": (1, 1)}


def _size_align(t, structs):
    if t.startswith("*"):
        return 8, 8
    m = re.match(r"\[(.*); (\d+)\]$", t)
    if m:
        s, a = _size_align(m.group(1), structs)
        return s * int(m.group(2)), a
    if t in _SIZES:
        return _SIZES[t]
    return _layout(structs[t], structs)[0:2]


def _layout(fields, structs):
    off, align, offs = 0, 1, []
    for _, t in fields:
        s, a = _size_align(t, structs)
        off = (off + a - 1) // a * a
        offs.append(off)
        off += s
        align = max(align, a)
    return (off + align - 1) // align * align, align, offs


def test_rust_layouts_equal_the_ctypes_mirror(parsed, rtm):
    _, r_st, _ = parsed["rust"]
    for name in ("rtm_sphere", "rtm_patch", "rtm_camera", "rtm_circle_plane", "rtm_capped_cylinder", "rtm_sdf",
                 "rtm_scene", "rtm_stats"):
        size, _, offs = _layout(r_st[name], r_st)
        ct = getattr(rtm.abi, name)
        assert size == C.sizeof(ct), name
        for (fname, _), off in zip(r_st[name], offs):
            cname = "type" if fname == "type_" else fname
            assert getattr(ct, cname).offset == off, (name, fname)


def test_crate_calls_only_bound_functions(parsed):
    _, _, r_fns = parsed["rust"]
    for f in ("rust/src/lib.rs", "rust/examples/closely_orbiting.rs", "rust/examples/closely_orbiting_seams.rs"):
        src = open(os.path.join(ROOT, f)).read()
        for n in set(re.findall(r"\b(rtm_[a-z0-9_]+)\s*\(", src)):
            assert n in r_fns, (f, n)
    ex = open(os.path.join(ROOT, "rust/examples/closely_orbiting.rs")).read()
    assert "render_frames" in ex  # the animation loop drives rtm_render_frames_async


def test_safe_layer_is_the_reference_surface():
    """The safe layer offers the reference's surface: the whole
    frame into host memory (Context::render over rtm_render_async + the copy) and one
    method per seam the reference's drivers call -- Viewport::rasterize (main.rs:445),
    processRaymarchingRays (main.rs:551), processRaytracingRays (main.rs:569) and
    renderColorImage (main.rs:710) -- each over its rtm_viewport_* call."""
    lib = open(os.path.join(ROOT, "rust/src/lib.rs")).read()
    seams = {"pub fn render(": "rtm_render_async(", "pub fn viewport(": "rtm_viewport_create(",
             "pub fn rasterize(": "rtm_viewport_rasterize(",
             "pub fn process_raymarching_rays(": "rtm_viewport_process_raymarching_rays(",
             "pub fn process_raytracing_rays(": "rtm_viewport_process_raytracing_rays(",
             "pub fn render_color_image(": "rtm_render_color_image(", "pub fn z_buffer(": "rtm_viewport_read_zbuffer("}
    for method, call in seams.items():
        i = lib.find(method)
        assert i >= 0, method
        body = lib[i:lib.find("\n    }", i) if method != "pub fn render_color_image(" else lib.find("\n}", i)]
        assert call in body, (method, call)
    assert "-> Result<Vec<f32>, Error>" in lib[lib.find("pub fn render("):lib.find("pub fn render(") + 300]
    assert "impl Drop for Viewport" in lib  # rtm_viewport_destroy
    ex = open(os.path.join(ROOT, "rust/examples/closely_orbiting_seams.rs")).read()
    for m in ("ctx.viewport(", ".rasterize(&scene)", ".process_raymarching_rays(", "render_color_image(&scene",
              "ctx.render(&scene"):
        assert m in ex, m
    # the north star's multi-GPU frame: Group over rtm_group_*, its
    # Drop bounding the wait before the communicators are destroyed
    group = {"pub fn new(": "rtm_group_create(", "pub fn render_into(": "rtm_group_render(",
             "pub fn set_host_direct(": "rtm_group_set_host_direct(",
             "pub fn set_partition(": "rtm_group_set_partition(", "pub fn synchronize(": "rtm_group_synchronize("}
    g0 = lib.find("impl Group {")
    assert g0 >= 0 and "pub struct Group" in lib
    for method, call in group.items():
        i = lib.find(method, g0)
        assert i >= 0, method
        assert call in lib[i:lib.find("\n    }", i)], (method, call)
    i = lib.find("pub fn render(", g0)
    assert "-> Result<Vec<u8>, Error>" in lib[i:i + 300] and "self.render_into(" in lib[i:lib.find("\n    }", i)]
    d = lib[lib.find("impl Drop for Group"):]
    d = d[:d.find("\n}")]
    assert d.find("rtm_group_synchronize(self.raw, self.drop_timeout_ms)") < d.find("rtm_group_destroy(self.raw)")
    ex = open(os.path.join(ROOT, "rust/examples/closely_orbiting_group.rs")).read()
    for m in ("Group::new(", "group.render_into(&scene", "RTM_FORMAT_RGB8", "for frame in 0..300"):
        assert m in ex, m
