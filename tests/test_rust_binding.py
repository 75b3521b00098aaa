"""CPU tier: the committed Rust binding (rust/verification/src/gpu/ffi.rs) declares exactly the C
ABI of include/zg.h, signature by signature. There is no cargo in the build image, so the
binding is checked textually: every function in the header has an `extern "C"` declaration with
the same name, the same number of parameters and C-compatible types in the same order, and the
same return type; the #define constants the binding mirrors have the same values; build.rs
compiles exactly the translation units zebra_amd/build.py does, for gfx950."""
import os
import re

from tests.conftest import ROOT

FFI = os.path.join(ROOT, "rust", "verification", "src", "gpu", "ffi.rs")
HDR = os.path.join(ROOT, "include", "zg.h")

# C type (normalised) -> Rust type
C2R = {"int": "c_int", "size_t": "usize", "uint64_t": "u64", "uint32_t": "u32", "void": None,
       "zg_ctx*": "*mut ZgCtx", "const zg_config*": "*const ZgConfig", "const char*": "*const c_char",
       "const uint8_t*": "*const u8", "uint8_t*": "*mut u8", "const void*": "*const c_void",
       "float*": "*mut f32", "double*": "*mut f64", "uint64_t*": "*mut u64", "const uint32_t*": "*const u32",
       "int*": "*mut c_int", "const int64_t*": "*const i64", "const uint64_t*": "*const u64",
       "size_t*": "*mut usize", "const size_t*": "*const usize"}


def c_decls():
    h = open(HDR).read()
    h = re.sub(r"/\*.*?\*/", "", h, flags=re.S)
    out = {}
    for m in re.finditer(r"^([A-Za-z_][\w\s\*]*?)\b(zg_\w+)\s*\(([^;]*?)\)\s*;", h, flags=re.M | re.S):
        ret, name, args = m.group(1).strip(), m.group(2), m.group(3).strip()
        params = []
        if args and args != "void":
            for a in args.split(","):
                a = " ".join(a.split())
                arr = "[" in a
                a = re.sub(r"\[.*?\]", "", a).strip()
                t = re.sub(r"\s*\b\w+$", "", a) if not a.endswith("*") else a   # drop the parameter name
                t = t.replace(" *", "*").replace("* ", "*").strip()
                if arr:
                    t += "*"
                params.append(t)
        out[name] = (" ".join(ret.split()).replace(" *", "*"), params)
    return out


def rust_decls():
    src = open(FFI).read()
    block = src[src.index('extern "C" {'):]
    out = {}
    for m in re.finditer(r"pub fn (zg_\w+)\s*\((.*?)\)\s*(?:->\s*([^;]+))?;", block, flags=re.S):
        name, args, ret = m.group(1), m.group(2), (m.group(3) or "").strip() or None
        params = [" ".join(a.split(":", 1)[1].split()) for a in args.split(",") if a.strip()]
        out[name] = (ret, params)
    return out


def test_every_header_function_is_bound_with_the_same_signature():
    c, r = c_decls(), rust_decls()
    assert len(c) >= 28
    assert sorted(c) == sorted(r), (set(c) ^ set(r))
    for name, (cret, cparams) in c.items():
        rret, rparams = r[name]
        assert C2R[cret] == rret, (name, cret, rret)
        assert len(cparams) == len(rparams), (name, cparams, rparams)
        for i, (ct, rt) in enumerate(zip(cparams, rparams)):
            assert C2R.get(ct) == rt, (name, i, ct, rt)


def test_constants_match_the_header():
    h = open(HDR).read()
    rs = open(FFI).read()
    defs = dict(re.findall(r"#define (ZG_\w+)\s+\(?(-?\d+)\)?", h))
    rdefs = dict(re.findall(r"pub const (ZG_\w+): \w+ = (-?\d+);", rs))
    assert len(rdefs) >= 25
    for k, v in rdefs.items():
        assert defs[k] == v, k


def test_config_struct_layout():
    h = open(HDR).read()
    body = re.search(r"typedef struct zg_config \{(.*?)\} zg_config;", h, re.S).group(1)
    cfields = [l.split(";")[0].split()[-1] for l in body.splitlines() if ";" in l]
    rs = open(FFI).read()
    rbody = re.search(r"pub struct ZgConfig \{(.*?)\n\}", rs, re.S).group(1)
    rfields = re.findall(r"pub (\w+):", rbody)
    assert cfields == rfields == ["device", "max_batch", "seeded", "seed"]


def test_build_rs_compiles_the_library_sources_for_gfx950():
    b = open(os.path.join(ROOT, "rust", "verification", "build.rs")).read()
    import runpy
    srcs = runpy.run_path(os.path.join(ROOT, "zebra_amd", "build.py"))["SOURCES"]
    rs = re.search(r"const SOURCES: \[&str; \d+\] =\s*\[(.*?)\];", b, re.S).group(1)
    assert re.findall(r'"([\w.]+)"', rs) == srcs
    assert "--offload-arch=gfx950" in b and "rustc-link-lib=dylib=zg" in b
    for f in re.findall(r'"([\w-]+\.json)"', b):
        assert os.path.exists(os.path.join(ROOT, "zebra_amd", "res", f))


def test_rust_module_layout_and_fallback():
    """the gpu module declares its submodules; the collector queues PHGR JoinSplits into one
    pghr13_verify call and has the GPU-error degradation path over the reference's own calls;
    the deferred writer mirrors zebra_amd/blocks_writer.py"""
    base = os.path.join(ROOT, "rust", "verification", "src", "gpu")
    mod = open(os.path.join(base, "mod.rs")).read()
    for m in ("collect", "cpu", "ffi", "writer"):
        assert "pub mod %s;" % m in mod and os.path.exists(os.path.join(base, m + ".rs"))
    col = open(os.path.join(base, "collect.rs")).read()
    assert "fn pghr13_verify" in col and "Plan::Pghr" in col and "prep_joinsplit_bn" in col
    assert "pub fn verify_block_or_cpu" in col and "impl Backend for GpuVerifier" in col
    cpu = open(os.path.join(base, "cpu.rs")).read()
    for call in ("verify_proof(", "Proof::<Bls12>::read(", "Pghr13Proof::from_raw(", "pghr13_verify(",
                 "redjubjub::PublicKey::<Bls12>::read("):
        assert call in cpu, call
    assert "oracle" not in cpu.replace("the test oracle", "")
    wr = open(os.path.join(base, "writer.rs")).read()
    assert "MAX_ORPHANED_BLOCKS: usize = 1024" in wr and "pub fn append_block" in wr and "pub fn flush" in wr
    # balanced delimiters in every Rust source (a cheap syntax sanity check without cargo)
    for f in ("mod.rs", "collect.rs", "cpu.rs", "ffi.rs", "writer.rs"):
        src = re.sub(r"//[^\n]*", "", open(os.path.join(base, f)).read())
        src = re.sub(r'"(\\.|[^"\\])*"', '""', src)
        for a, b in ("()", "[]", "{}"):
            assert src.count(a) == src.count(b), (f, a)
