"""INTEGRATION.md's Rust binding against the C headers (CPU only).

rustc is not in this image, so nothing compiles the `extern "C"` block a crate
maintainer would paste.  This test is its guard: it
parses every prototype of include/msw.h and include/msw_fastq.h and every
`pub fn` of the block, and requires the same set of names and, per function,
the same arity, argument types and return type -- integer widths and
signedness, pointer depth and const/mut -- plus every `#[repr(C)]` struct
field by field against its C typedef.  A missing or mistyped entry fails.
The reference's boundary this replaces is the loader callback and the
gpu_align call (smith_waterman/src/aligner.rs:107-108, :410).
"""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("msw.h", "msw_fastq.h")]
INTEGRATION = os.path.join(ROOT, "INTEGRATION.md")

# C base type -> canonical; Rust base type -> canonical
C_BASE = {"int": "i32", "int32_t": "i32", "unsigned": "u32", "uint32_t": "u32", "uint64_t": "u64",
          "int64_t": "i64", "size_t": "usize", "int16_t": "i16", "uint16_t": "u16", "uint8_t": "u8",
          "char": "c_char", "double": "f64", "void": "void"}
RUST_BASE = {"c_int": "i32", "i32": "i32", "u32": "u32", "u64": "u64", "i64": "i64", "usize": "usize",
             "i16": "i16", "u16": "u16", "u8": "u8", "c_char": "c_char", "f64": "f64", "c_void": "void"}


def _strip_c(text):
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    text = re.sub(r"//[^\n]*", " ", text)
    return "\n".join(l for l in text.splitlines() if not l.lstrip().startswith("#"))


def c_type(decl):
    """'const uint8_t* s1' / 'msw_ctx** out' / 'int' -> canonical type tuple."""
    decl = decl.replace("*", " * ").split()
    if decl and decl[-1] not in C_BASE and decl[-1] != "*" and len(decl) > 1:
        decl = decl[:-1]  # drop the parameter name
    const = "const" in decl[:2]
    words = [w for w in decl if w not in ("const", "struct")]
    stars = words.count("*")
    base = [w for w in words if w != "*"]
    assert len(base) == 1, decl
    t = C_BASE.get(base[0], base[0])
    for k in range(stars):
        # only the pointee of the innermost pointer carries a leading const
        t = ("ptr", "const" if (k == 0 and const) else "mut", t)
    return t


def rust_type(s):
    s = s.strip()
    m = re.match(r"^\*(const|mut)\s+(.*)$", s)
    if m:
        return ("ptr", m.group(1), rust_type(m.group(2)))
    m = re.match(r"^\[\s*(\w+)\s*;\s*(\d+)\s*\]$", s)
    if m:
        return ("array", RUST_BASE.get(m.group(1), m.group(1)), int(m.group(2)))
    return RUST_BASE.get(s, s)


def c_functions():
    out = {}
    for h in HEADERS:
        text = _strip_c(open(h).read())
        for ret, name, params in re.findall(r"([A-Za-z_][\w \t\*]*?)\b(msw_\w+)\s*\(([^;{}()]*)\)\s*;", text):
            ret = ret.strip()
            if ret.startswith("typedef"):
                continue
            ps = [p.strip() for p in params.split(",") if p.strip()]
            if ps == ["void"]:
                ps = []
            out[name] = (c_type(ret), [c_type(p) for p in ps])
    return out


def c_structs():
    out = {}
    for h in HEADERS:
        text = _strip_c(open(h).read())
        for body, name in re.findall(r"typedef\s+struct\s*\{(.*?)\}\s*(\w+)\s*;", text, flags=re.S):
            fields = []
            for f in body.split(";"):
                f = " ".join(f.split())
                if not f:
                    continue
                m = re.match(r"^(.*?)(\w+)\s*\[(\d+)\]$", f)
                if m:
                    fields.append((m.group(2), ("array", C_BASE[m.group(1).strip()], int(m.group(3)))))
                    continue
                for part in _split_decl(f):
                    fields.append(part)
            out[name] = fields
    return out


def _split_decl(f):
    """'uint32_t min_len, max_len' -> [(min_len, u32), (max_len, u32)]."""
    first, *rest = [x.strip() for x in f.split(",")]
    m = re.match(r"^(.*?)(\w+)$", first)
    base, name = m.group(1).strip(), m.group(2)
    res = [(name, c_type(base + " " + name))]
    for r in rest:
        res.append((r, c_type(base + " " + r)))
    return res


def rust_code():
    text = open(INTEGRATION).read()
    return "\n".join(re.findall(r"```rust\n(.*?)```", text, flags=re.S))


def rust_functions():
    code = rust_code()
    blocks = re.findall(r'extern\s+"C"\s*\{(.*?)\n\}', code, flags=re.S)
    assert blocks, "no extern \"C\" block in INTEGRATION.md"
    out = {}
    for blk in blocks:
        blk = re.sub(r"//[^\n]*", " ", blk)
        for name, params, ret in re.findall(r"pub\s+fn\s+(msw_\w+)\s*\(([^)]*)\)\s*(?:->\s*([^;]+))?;", blk):
            ps = []
            for p in params.split(","):
                p = p.strip()
                if not p:
                    continue
                _, t = p.split(":", 1)
                ps.append(rust_type(t))
            assert name not in out, f"{name} declared twice"
            out[name] = (rust_type(ret) if ret.strip() else "void", ps)
    return out


def rust_structs():
    out = {}
    for name, body in re.findall(r"pub\s+struct\s+(\w+)\s*\{(.*?)\}", rust_code(), flags=re.S):
        fields = []
        for f in re.findall(r"(?:pub\s+)?(\w+)\s*:\s*([^,]+?)\s*(?:,|$)", body.strip()):
            fields.append((f[0], rust_type(f[1])))
        out[name] = fields
    return out


def test_every_export_is_bound():
    c, r = c_functions(), rust_functions()
    assert len(c) >= 45, sorted(c)
    missing = sorted(set(c) - set(r))
    extra = sorted(set(r) - set(c))
    assert not missing, f"INTEGRATION.md's extern block lacks {missing}"
    assert not extra, f"INTEGRATION.md binds functions the headers do not declare: {extra}"


@pytest.mark.parametrize("name", sorted(c_functions()))
def test_signature_matches(name):
    c_ret, c_args = c_functions()[name]
    r = rust_functions().get(name)
    assert r is not None, f"{name} missing from the Rust block"
    r_ret, r_args = r
    assert len(r_args) == len(c_args), f"{name}: arity {len(r_args)} in Rust, {len(c_args)} in C"
    for k, (a, b) in enumerate(zip(c_args, r_args)):
        assert a == b, f"{name} argument {k}: C {a} vs Rust {b}"
    assert c_ret == r_ret, f"{name} return: C {c_ret} vs Rust {r_ret}"


def test_structs_match():
    cs, rs = c_structs(), rust_structs()
    for name, cf in cs.items():
        assert name in rs, f"struct {name} missing from INTEGRATION.md"
        rf = rs[name]
        assert len(rf) == len(cf), f"{name}: {len(rf)} fields in Rust, {len(cf)} in C"
        for (cn, ct), (rn, rt) in zip(cf, rf):
            assert cn == rn.rstrip("_"), f"{name}: field {cn} vs {rn}"
            assert ct == rt, f"{name}.{cn}: C {ct} vs Rust {rt}"


def test_parser_catches_a_mistyped_entry(monkeypatch):
    """The guard itself: a u32 where the header says u64 is caught."""
    code = rust_code().replace("n: u64, wins: *mut u8, win_stride: u32", "n: u32, wins: *mut u8, win_stride: u32")
    assert code != rust_code()
    monkeypatch.setattr(__import__(__name__), "rust_code", lambda: code)
    c_ret, c_args = c_functions()["msw_genome_cut_device"]
    assert rust_functions()["msw_genome_cut_device"][1] != c_args
