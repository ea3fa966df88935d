"""CPU: the Rust drop-in shim (rust/rlnc-hip, the files a maintainer adds to the reference crate) agrees with the C
ABI it binds.  There is no cargo/rustc in this image, so the check is textual: every function and struct of
include/rlnc_hip.h is declared in src/hip/ffi.rs with the same name, argument count and C types (pointer depth and
constness, size_t = usize, int = c_int, ...), the status constants agree, mod.rs maps every RLNCError code to its
variant in errors.rs order without cloning (RLNCError derives only Debug + PartialEq, reference errors.rs:2), and
the crate patch applies to the reference (when it is present)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "rust", "rlnc-hip")
FFI = os.path.join(SHIM, "src", "hip", "ffi.rs")
MOD = os.path.join(SHIM, "src", "hip", "mod.rs")
HEADER = os.path.join(ROOT, "include", "rlnc_hip.h")

_C_BASE = {"uint8_t": "u8", "int32_t": "i32", "int64_t": "i64", "uint64_t": "u64", "size_t": "usize", "int": "c_int",
           "char": "c_char", "void": "c_void"}
_RS_BASE = {"u8", "i32", "i64", "u64", "usize", "c_int", "c_char", "c_void"}


def _strip_c_comments(txt):
    txt = re.sub(r"/\*.*?\*/", " ", txt, flags=re.S)
    return re.sub(r"//[^\n]*", " ", txt)


def _c_type(decl):
    """'const uint8_t *' -> ('ptr', 'const', 'u8'); 'rlnc_context **' -> ('ptr', 'mut', ('ptr', 'mut', ...)).
    Pointer constness follows C: the qualifier left of the base (or right of it, before the first '*') applies to
    the pointee of the innermost pointer."""
    decl = decl.strip()
    stars = decl.count("*")
    base = decl.replace("*", " ").split()
    const = "const" in base
    base = [w for w in base if w not in ("const", "struct")]
    assert len(base) == 1, decl
    t = _C_BASE.get(base[0], base[0])
    if stars == 0:
        return t
    t = ("ptr", "const" if const else "mut", t)
    for _ in range(stars - 1):
        t = ("ptr", "mut", t)
    return t


def _rs_type(decl):
    decl = decl.strip()
    m = re.match(r"\*(const|mut)\s+(.*)$", decl)
    if m:
        return ("ptr", m.group(1), _rs_type(m.group(2)))
    assert re.fullmatch(r"\w+|\[u8; 0\]", decl), decl
    return decl


def header_api():
    txt = _strip_c_comments(open(HEADER).read())
    funcs = {}
    for m in re.finditer(r"^\s*([A-Za-z_][\w\s\*]*?[\s\*])(rlnc_\w+)\s*\(([^)]*)\)\s*;", txt, flags=re.M):
        ret, name, args = m.group(1), m.group(2), m.group(3).strip()
        ret = ret.replace("typedef", "").strip()
        params = []
        if args and args != "void":
            for a in args.split(","):
                a = re.sub(r"\[\d*\]", "*", a.strip())  # array parameters decay to pointers
                pm = re.match(r"(.*?)(\w+)$", a)
                params.append(_c_type(pm.group(1)))
        funcs[name] = ("void" if ret == "void" else _c_type(ret), params)
    structs = {}
    for m in re.finditer(r"typedef\s+struct\s+(\w+)\s*\{(.*?)\}\s*\w+\s*;", txt, flags=re.S):
        fields = []
        for decl in m.group(2).split(";"):
            decl = decl.strip()
            if not decl:
                continue
            dm = re.match(r"((?:const\s+)?\w+)\s*(.*)$", decl)
            base = dm.group(1)
            for d in dm.group(2).split(","):
                d = d.strip()
                stars = d.count("*")
                fname = d.replace("*", "").strip()
                fields.append((fname, _c_type(base + " " + "*" * stars)))
        structs[m.group(1)] = fields
    consts = dict((n, int(v)) for n, v in re.findall(r"#define\s+(RLNC_\w+)\s+(\d+)", open(HEADER).read()))
    return funcs, structs, consts


def ffi_api():
    txt = re.sub(r"//[^\n]*", " ", open(FFI).read())
    blocks = re.findall(r"(unsafe\s+)?extern\s+\"C\"\s*\{(.*?)\n\}", txt, flags=re.S)
    assert len(blocks) == 1, "exactly one extern block"
    assert blocks[0][0].strip() == "unsafe", "edition 2024 (reference Cargo.toml:4) requires `unsafe extern`"
    funcs = {}
    for m in re.finditer(r"pub\s+fn\s+(\w+)\s*\((.*?)\)\s*(->\s*([^;]+))?;", blocks[0][1], flags=re.S):
        name, args, ret = m.group(1), m.group(2), m.group(4)
        params = []
        for a in [x.strip() for x in args.split(",") if x.strip()]:
            pname, ptype = a.split(":", 1)
            params.append(_rs_type(ptype))
        funcs[name] = ("void" if ret is None else _rs_type(ret.strip()), params)
    structs = {}
    for m in re.finditer(r"#\[repr\(C\)\]\s*(?:#\[derive\([^)]*\)\]\s*)?pub\s+struct\s+(\w+)\s*\{(.*?)\}", txt, flags=re.S):
        fields = []
        for f in [x.strip() for x in m.group(2).split(",") if x.strip()]:
            fname, ftype = f.split(":", 1)
            fname = fname.replace("pub", "").strip()
            fields.append((fname, _rs_type(ftype)))
        structs[m.group(1)] = fields
    consts = dict((n, int(v)) for n, v in re.findall(r"pub\s+const\s+(RLNC_\w+)\s*:\s*c_int\s*=\s*(\d+)\s*;", txt))
    return funcs, structs, consts


def test_every_header_function_is_bound_with_the_same_signature():
    hf, _, _ = header_api()
    rf, _, _ = ffi_api()
    assert len(hf) >= 60
    assert sorted(hf) == sorted(rf), (sorted(set(hf) - set(rf)), sorted(set(rf) - set(hf)))
    for name, (ret, params) in hf.items():
        rret, rparams = rf[name]
        assert len(params) == len(rparams), (name, params, rparams)
        assert ret == rret, (name, ret, rret)
        for i, (c, r) in enumerate(zip(params, rparams)):
            assert c == r, (name, i, c, r)


def test_header_symbols_match_the_library_table():
    from rlnc_amd import _lib

    hf, _, _ = header_api()
    assert sorted(hf) == _lib.header_symbols()


def test_descriptor_structs_have_the_same_layout():
    _, hs, _ = header_api()
    _, rs, _ = ffi_api()
    for name, fields in hs.items():
        assert name in rs, name
        rfields = rs[name]
        assert len(fields) == len(rfields), name
        for (cn, ct), (rn, rt) in zip(fields, rfields):
            assert ct == rt, (name, cn, ct, rt)
            assert cn == rn or (cn, rn) == ("in", "in_"), (name, cn, rn)  # `in` is a Rust keyword
    opaque = {"rlnc_context", "rlnc_encoder", "rlnc_decoder", "rlnc_recoder", "rlnc_elimination"}
    assert opaque <= set(rs)
    assert all(rs[o] == [("_p", "[u8; 0]")] for o in opaque)


def test_status_constants_agree():
    _, _, hc = header_api()
    _, _, rc = ffi_api()
    assert hc == rc


def test_status_mapping_follows_errors_rs_order_without_clone():
    from rlnc_amd.errors import STATUS_NAMES

    src = open(MOD).read()
    _, _, rc = ffi_api()
    arms = dict(re.findall(r"ffi::(RLNC_ERR_\w+)\s*=>\s*Err\(RLNCError::(\w+)\)", src))
    assert len(arms) == 13
    for const, variant in arms.items():
        assert STATUS_NAMES[rc[const]] == variant, (const, variant)
    assert ".clone()" not in re.sub(r"//[^\n]*", "", src.split("fn status")[1].split("\n}\n")[0])


def test_reference_signatures_are_kept():
    """The public methods a user of rlnc::full calls keep the reference's signatures (encoder.rs:27-269,
    decoder.rs:25-177, recoder.rs:26-171)."""
    src = re.sub(r"\s+", " ", open(MOD).read())
    want = [
        "pub fn new(data: Vec<u8>, piece_count: usize) -> Result<Encoder, RLNCError>",
        "pub fn code_with_buf<R: Rng + ?Sized>(&self, rng: &mut R, full_coded_piece: &mut [u8]) -> Result<(), RLNCError>",
        "pub fn code<R: Rng + ?Sized>(&self, rng: &mut R) -> Vec<u8>",
        "pub fn new(piece_byte_len: usize, required_piece_count: usize) -> Result<Decoder, RLNCError>",
        "pub fn decode(&mut self, full_coded_piece: &[u8]) -> Result<(), RLNCError>",
        "pub fn is_already_decoded(&self) -> bool",
        "pub fn get_decoded_data(self) -> Result<Vec<u8>, RLNCError>",
        "pub fn new(data: Vec<u8>, full_coded_piece_byte_len: usize, num_pieces_coded_together: usize) -> Result<Recoder, RLNCError>",
        "pub fn recode_with_buf<R: Rng + ?Sized>(&mut self, rng: &mut R, full_recoded_piece: &mut [u8]) -> Result<(), RLNCError>",
        "pub fn recode<R: Rng + ?Sized>(&mut self, rng: &mut R) -> Vec<u8>",
    ]
    for w in want:
        assert w in src, w
    for getter in ["get_piece_count", "get_piece_byte_len", "get_full_coded_piece_byte_len",
                   "get_num_pieces_coded_together", "get_received_piece_count", "get_useful_piece_count",
                   "get_remaining_piece_count", "get_original_num_pieces_coded_together",
                   "get_num_pieces_recoded_together"]:
        assert f"pub fn {getter}(&self) -> usize" in src, getter


REF = "/root/reference"


@pytest.mark.skipif(not os.path.isdir(REF) or shutil.which("patch") is None, reason="reference crate not present")
def test_crate_patch_applies_to_the_reference(tmp_path):
    dst = tmp_path / "rlnc"
    shutil.copytree(REF, dst, ignore=shutil.ignore_patterns(".git", "target", "plots"))
    subprocess.run(["patch", "-p1", "-i", os.path.join(SHIM, "reference.patch")], cwd=dst, check=True,
                   capture_output=True)
    lib = (dst / "src" / "lib.rs").read_text()
    assert '#[cfg(feature = "hip")]\nmod hip;' in lib
    full = (dst / "src" / "full" / "mod.rs").read_text()
    assert "pub use crate::hip::{Decoder, Encoder, Recoder};" in full
    assert "hip = []" in (dst / "Cargo.toml").read_text()
    # every crate-level name the shim uses exists in the patched crate
    assert "pub use crate::common::errors::RLNCError;" in lib
    errors = (dst / "src" / "common" / "errors.rs").read_text()
    assert "#[derive(Debug, PartialEq)]" in errors  # not Clone: the shim must not clone variants
