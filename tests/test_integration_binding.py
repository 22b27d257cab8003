"""The Rust binding in INTEGRATION.md (the reference-side `extern "C"` block a
crate maintainer would add, replacing Writer::spill_block,
src/table/writer/mod.rs:303-337, and Scanner, src/table/scanner.rs:50-92)
against include/lsmgpu.h: the same functions, and for each the same number of
parameters with the same C types (mapped to their Rust FFI spelling) and the
same return type.  CPU only: no cargo/rustc in this image, so this is the
mechanical check that the binding has not drifted from the header."""
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent

C_TO_RUST = {
    "int": "c_int", "size_t": "usize", "float": "f32",
    "uint8_t": "u8", "uint16_t": "u16", "uint32_t": "u32", "uint64_t": "u64",
    "int32_t": "i32", "int64_t": "i64", "char": "c_char", "void": "c_void",
    "lsm_items": "LsmItems", "lsm_items32": "LsmItems32", "lsm_parsed_items": "LsmParsedItems", "lsm_parsed_items16": "LsmParsedItems16",
    "lsm_block_params": "LsmBlockParams", "lsm_decode_tuning": "LsmDecodeTuning",
    "lsm_point_result": "LsmPointResult", "lsm_table_scan": "LsmTableScan",
}


def c_type_to_rust(t):
    t = " ".join(t.split())
    m = re.fullmatch(r"(const\s+)?(\w+)\s*(\*?)", t)
    assert m, t
    const, base, star = m.groups()
    r = C_TO_RUST[base]
    if star:
        return ("*const " if const else "*mut ") + r
    return r


def header_functions():
    text = (ROOT / "include" / "lsmgpu.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"#.*", "", text)
    out = {}
    for m in re.finditer(r"([\w\s\*]+?)\b(lsm_\w+)\s*\(([^)]*)\)\s*;", text):
        ret, name, params = m.group(1), m.group(2), m.group(3)
        ret = ret.strip().split("\n")[-1].strip()
        plist = [] if params.strip() in ("", "void") else [p.strip() for p in params.split(",")]
        types = []
        for p in plist:
            pm = re.fullmatch(r"(.*?)(\w+)", " ".join(p.split()))
            types.append(c_type_to_rust(pm.group(1).strip()))
        out[name] = (c_type_to_rust(ret), types)
    return out


def rust_type(t):
    t = " ".join(t.split())
    t = re.sub(r"\*\s*(const|mut)\s+", r"*\1 ", t)
    return t


def binding_functions():
    text = (ROOT / "INTEGRATION.md").read_text()
    blocks = re.findall(r"extern \"C\" \{(.*?)\n\}", text, flags=re.S)
    assert len(blocks) == 1, "INTEGRATION.md holds one extern \"C\" block"
    body = re.sub(r"//[^\n]*", "", blocks[0])
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    out = {}
    for m in re.finditer(r"pub fn (lsm_\w+)\s*\(([^)]*)\)\s*(?:->\s*([^;]+))?;", body, flags=re.S):
        name, params, ret = m.group(1), m.group(2), m.group(3)
        types = []
        for p in [p for p in params.split(",") if p.strip()]:
            _, ty = p.split(":", 1)
            types.append(rust_type(ty))
        out[name] = (rust_type(ret) if ret else "()", types)
    return out


def test_binding_names_match_header():
    h, b = header_functions(), binding_functions()
    assert set(h) == set(b), (sorted(set(h) - set(b)), sorted(set(b) - set(h)))


def test_binding_signatures_match_header():
    h, b = header_functions(), binding_functions()
    for name, (ret, params) in h.items():
        bret, bparams = b[name]
        assert len(bparams) == len(params), (name, len(bparams), len(params))
        assert bparams == params, (name, bparams, params)
        assert bret == ret, (name, bret, ret)


def test_binding_abi_version_note():
    text = (ROOT / "INTEGRATION.md").read_text()
    ver = int(re.search(r"#define LSM_ABI_VERSION (\d+)", (ROOT / "include" / "lsmgpu.h").read_text()).group(1))
    assert f"`LSM_ABI_VERSION` {ver}" in text
