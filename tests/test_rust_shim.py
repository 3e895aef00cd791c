"""The Rust shim crate (rust/backuwup-gpu) against the C ABI it binds, without a Rust toolchain.

There is no rustc in this image, so the crate is not compiled here.  This test reads its
`extern "C"` block and `#[repr(C)]` structs as text and checks them against include/backuwup_gpu.h (and the
backuwup_gpu_pack.h it includes):
every function the header declares is bound once, with the same name, arity, return type, and per
argument the same pointer depth, constness of the pointee and integer width; every struct has the
same fields in the same order with the same types.  The reference call sites it replaces are
dir_packer.rs:254-266 (FastCDC::new + iterator) and :286 (blake3::hash)."""
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
HEADERS = [os.path.join(ROOT, "include", h) for h in ("backuwup_gpu.h", "backuwup_gpu_pack.h")]
CRATE = os.path.join(ROOT, "rust", "backuwup-gpu")

C_BASE = {"int": "i32", "uint8_t": "u8", "uint32_t": "u32", "uint64_t": "u64", "char": "i8", "double": "f64",
          "void": "void"}
R_BASE = {"c_int": "i32", "i32": "i32", "u8": "u8", "u32": "u32", "u64": "u64", "c_char": "i8", "i8": "i8",
          "f64": "f64", "c_void": "void", "()": "void"}


def _header_text():
    return "\n".join(open(h).read() for h in HEADERS)


def _strip_c_comments(txt):
    return re.sub(r"//[^\n]*", "", re.sub(r"/\*.*?\*/", "", txt, flags=re.S))


def c_type(decl, has_name=True):
    """'const uint8_t* src' / 'uint8_t out[32]' / 'bw_ctx** out' -> (depth, const_pointee, base)."""
    d = decl.strip()
    depth = 0
    if "[" in d:  # an array parameter is a pointer
        depth += 1
        d = d[:d.index("[")]
    const = d.startswith("const ")
    if const:
        d = d[len("const "):]
    depth += d.count("*")
    toks = d.replace("*", " ").split()
    if has_name:
        toks = toks[:-1]
    assert len(toks) == 1, decl
    return depth, const and depth > 0, C_BASE.get(toks[0], toks[0])


def r_type(t):
    """'*mut *const u8' -> (2, True, 'u8'); 'c_int' -> (0, False, 'i32')."""
    t = t.strip()
    quals = re.findall(r"\*(const|mut)\s*", t)
    base = re.sub(r"\*(const|mut)\s*", "", t).strip()
    if base.startswith("std::os::raw::"):
        base = base[len("std::os::raw::"):]
    return len(quals), bool(quals) and quals[-1] == "const", R_BASE.get(base, base)


def header_functions():
    txt = _strip_c_comments(_header_text())
    out = {}
    for m in re.finditer(r"^\s*((?:const\s+)?(?:int|void|char|uint\w+)\s*\*?)\s*(bw_\w+)\s*\(([^)]*)\)\s*;", txt,
                         re.M | re.S):
        ret = c_type(m.group(1), has_name=False)
        params = [p for p in (x.strip() for x in m.group(3).split(",")) if p and p != "void"]
        out[m.group(2)] = (ret, [c_type(p) for p in params])
    return out


def header_structs():
    txt = _strip_c_comments(_header_text())
    out = {}
    for m in re.finditer(r"typedef\s+struct\s+(\w+)\s*\{(.*?)\}\s*(\w+)\s*;", txt, re.S):
        fields = []
        for line in m.group(2).split(";"):
            line = " ".join(line.split())
            if not line:
                continue
            const = line.startswith("const ")
            if const:
                line = line[len("const "):]
            line = line.replace("*", " * ")
            head, names = line.split(" ", 1)
            for nm in names.split(","):
                nm = nm.strip()
                depth = nm.count("*")
                nm = nm.replace("*", "").strip()
                arr = re.match(r"(\w+)\[(\d+)\]", nm)
                base = C_BASE.get(head, head)
                if arr:
                    fields.append((arr.group(1), ("arr", base, int(arr.group(2)))))
                else:
                    fields.append((nm, (depth, const and depth > 0, base)))
        out[m.group(3)] = fields
    return out


def crate_source():
    return open(os.path.join(CRATE, "src", "lib.rs")).read()


def rust_functions():
    src = crate_source()
    block = re.search(r'extern "C"\s*\{(.*?)\n    \}', src, re.S)
    assert block, "no extern \"C\" block in src/lib.rs"
    body = re.sub(r"//[^\n]*", "", block.group(1))
    out = {}
    for m in re.finditer(r"pub fn (bw_\w+)\s*\((.*?)\)\s*(?:->\s*([^;]+))?;", body, re.S):
        name, args, ret = m.group(1), m.group(2), m.group(3)
        params = []
        for a in (x.strip() for x in args.split(",")):
            if a:
                params.append(r_type(a.split(":", 1)[1]))
        assert name not in out, "bound twice: " + name
        out[name] = (r_type(ret) if ret else (0, False, "void"), params)
    return out


def rust_structs():
    src = crate_source()
    out = {}
    for m in re.finditer(r"#\[repr\(C\)\]\s*(?:#\[derive\([^)]*\)\]\s*)?pub struct (bw_\w+)\s*\{(.*?)\}", src, re.S):
        fields = []
        for f in re.finditer(r"(?:pub\s+)?(\w+):\s*([^,]+),", m.group(2)):
            nm, t = f.group(1), f.group(2).strip()
            arr = re.match(r"\[(\w+);\s*(\d+)\]", t)
            if arr:
                fields.append((nm, ("arr", R_BASE.get(arr.group(1), arr.group(1)), int(arr.group(2)))))
            else:
                fields.append((nm, r_type(t)))
        out[m.group(1)] = [f for f in fields if f[0] != "_private"]
    return out


def test_crate_files_present():
    for f in ("Cargo.toml", "build.rs", os.path.join("src", "lib.rs")):
        assert os.path.isfile(os.path.join(CRATE, f)), f
    toml = open(os.path.join(CRATE, "Cargo.toml")).read()
    assert 'links = "backuwup_amd"' in toml
    assert "rustc-link-lib=dylib=backuwup_amd" in open(os.path.join(CRATE, "build.rs")).read()


def test_every_header_function_bound_with_matching_signature():
    c, r = header_functions(), rust_functions()
    assert len(c) > 60
    missing = sorted(set(c) - set(r))
    extra = sorted(set(r) - set(c))
    assert not missing and not extra, (missing, extra)
    for name, (cret, cparams) in c.items():
        rret, rparams = r[name]
        assert rret == cret, (name, "return", rret, cret)
        assert len(rparams) == len(cparams), (name, "arity", len(rparams), len(cparams))
        for k, (rp, cp) in enumerate(zip(rparams, cparams)):
            assert rp == cp, (name, "argument %d" % k, rp, cp)


def test_structs_match_header():
    c, r = header_structs(), rust_structs()
    for name in ("bw_chunk", "bw_blob", "bw_params", "bw_tree", "bw_tree_blob", "bw_packfile", "bw_index_file"):
        assert name in c and name in r, name
        assert r[name] == c[name], (name, r[name], c[name])


def test_host_transport_typedef_matches():
    """bw_host_all_to_all: int (*)(void* user, const void* send, void* recv, uint64_t bytes_per_rank)."""
    txt = _strip_c_comments(_header_text())
    m = re.search(r"typedef\s+int\s*\(\s*\*\s*bw_host_all_to_all\s*\)\s*\(([^)]*)\)\s*;", txt)
    cparams = [c_type(p) for p in m.group(1).split(",")]
    src = crate_source()
    rm = re.search(r"pub type bw_host_all_to_all\s*=\s*Option<unsafe extern \"C\" fn\((.*?)\)\s*->\s*c_int>", src, re.S)
    assert rm
    rparams = [r_type(a.split(":", 1)[1]) for a in rm.group(1).split(",") if a.strip()]
    assert rparams == cparams


def test_drop_ins_mirror_the_crates():
    """The names backuwup imports: fastcdc::v2020::{FastCDC, Chunk} with FastCDC::new(&[u8], u32, u32, u32)
    and Chunk { hash: u64, offset: usize, length: usize }; blake3::hash(&[u8]) -> Hash, Hash: Into<[u8; 32]>."""
    src = crate_source()
    assert re.search(r"pub fn new\(source: &'a \[u8\], min_size: u32, avg_size: u32, max_size: u32\) -> Self", src)
    assert re.search(r"pub struct Chunk \{\s*pub hash: u64,\s*pub offset: usize,\s*pub length: usize,\s*\}", src)
    assert re.search(r"impl Iterator for FastCDC<'_> \{\s*type Item = Chunk;", src)
    assert re.search(r"pub fn hash\(input: &\[u8\]\) -> Hash", src)
    assert "impl From<Hash> for [u8; 32]" in src


def test_checker_catches_drift(monkeypatch):
    """The comparison is not vacuous: a narrowed integer or a lost const is seen."""
    import sys
    mod = sys.modules[__name__]
    src = crate_source()
    c = header_functions()
    for old, new, fn in [("src: *const u8, len: u64, min_size", "src: *const u8, len: u32, min_size", "bw_fastcdc_chunks"),
                         ("prk: *const u8, d_src: *const u8", "prk: *mut u8, d_src: *const u8", "bw_seal_device")]:
        assert old in src
        monkeypatch.setattr(mod, "crate_source", lambda s=src.replace(old, new, 1): s)
        assert rust_functions()[fn] != c[fn]
    monkeypatch.setattr(mod, "crate_source", lambda: src)
