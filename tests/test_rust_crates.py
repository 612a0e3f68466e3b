"""The Rust binding a neptune-core maintainer would add (neptune-core_amd/rust/): the -sys crate
declares every entry point of include/neptune_hip.h, with the same argument count, and mirrors the
POD structs field for field.  No Rust toolchain exists in this container, so this is a text check
of the sources (the ABI itself is exercised by the Python and C99 tests)."""
import os
import re

from test_capi_symbols import declared_symbols

ROOT = os.path.join(os.path.dirname(__file__), "..")
SYS = os.path.join(ROOT, "neptune-core_amd", "rust", "neptune-hip-sys", "src", "lib.rs")
SAFE = os.path.join(ROOT, "neptune-core_amd", "rust", "neptune-hip", "src", "lib.rs")


def _header():
    return re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "neptune_hip.h")).read(), flags=re.S)


def _rust_fns():
    src = open(SYS).read()
    return {m.group(1): m.group(2) for m in re.finditer(r"pub fn (nhip_[a-z0-9_]+)\(([^)]*)\)", src, flags=re.S)}


def test_sys_crate_declares_every_symbol_with_its_arity():
    fns = _rust_fns()
    assert set(fns) == declared_symbols()
    hdr = _header()
    for name, args in fns.items():
        c = re.search(rf"\b{name}\s*\(([^;]*?)\)\s*;", hdr, flags=re.S).group(1).strip()
        c_arity = 0 if c in ("", "void") else c.count(",") + 1
        r_arity = 0 if not args.strip() else args.count(",") + 1
        assert c_arity == r_arity, name


def _c_struct_fields(name):
    body = re.search(r"typedef struct \{([^{}]*?)\}\s*" + name + ";", _header(), flags=re.S).group(1)
    fields = []
    for decl in body.split(";"):
        decl = decl.strip()
        if not decl:
            continue
        names = decl.split(None, 1)[1] if not decl.startswith("const") else decl.split(None, 2)[2]
        for n in names.split(","):
            fields.append(re.sub(r"[\s*]|\[.*\]", "", n))
    return fields


def _rust_struct_fields(name):
    body = re.search(r"pub struct " + name + r" \{(.*?)\n\}", open(SYS).read(), flags=re.S).group(1)
    return re.findall(r"pub ([a-z0-9_]+):", body)


def test_sys_structs_mirror_the_header():
    for s in ("nhip_stark_params", "nhip_claim", "nhip_proof", "nhip_stats", "nhip_queue_profile", "nhip_blk_block",
              "nhip_tx", "nhip_pow_mast_paths"):
        assert _rust_struct_fields(s) == _c_struct_fields(s), s


def test_safe_crate_covers_the_drop_in_surface():
    src = open(SAFE).read()
    for must in ("pub fn verify(&self, claim: &Claim, proof: &Proof)", "pub fn verify_batch(&self, items: &[(Claim, Proof)])",
                 "pub struct GpuNode", "nhip_group_verify_batch", "nhip_queue_verify", "pub fn verify_or_cpu",
                 "triton_vm::verify(Stark::default()"):
        assert must in src, must
    for f in ("Cargo.toml", "build.rs"):
        assert os.path.exists(os.path.join(ROOT, "neptune-core_amd", "rust", "neptune-hip-sys", f))
    assert os.path.exists(os.path.join(ROOT, "neptune-core_amd", "rust", "neptune-hip", "Cargo.toml"))


def test_air_exporter_matches_the_python_mirror_and_the_descriptor_format():
    """rust/neptune-hip/src/air_export.rs (not compiled here) and its Python mirror
    neptune_hip.air_export (tested against the oracle in tests/test_air_export.py) use the same
    descriptor constants and handle the same node kinds; the process-wide init is exported."""
    from neptune_hip import air_export as E
    src = open(os.path.join(ROOT, "neptune-core_amd", "rust", "neptune-hip", "src", "air_export.rs")).read()
    consts = {m.group(1): int(m.group(2).replace("_", ""), 0)
              for m in re.finditer(r"pub const ([A-Z_]+): u64 = (0x[0-9a-fA-F_]+|\d+);", src)}
    for name in ("AIR_MAGIC", "OP_INPUT", "OP_CONST", "OP_ADD", "OP_MUL", "IN_MAIN_CURR", "IN_AUX_CURR",
                 "IN_MAIN_NEXT", "IN_AUX_NEXT", "IN_CHALLENGE"):
        assert consts[name] == getattr(E, name), name
    for kind in ("BConst", "XConst", "Input", "Challenge", "BinOp"):
        assert f"CircuitExpression::{kind}" in src, kind
    for ind in ("SingleRowIndicator::Main", "SingleRowIndicator::Aux", "DualRowIndicator::CurrentMain",
                "DualRowIndicator::CurrentAux", "DualRowIndicator::NextMain", "DualRowIndicator::NextAux"):
        assert ind in src, ind
    assert "ExportError::UnknownNode" in src and "Challenges::SAMPLE_COUNT" in src
    safe = open(SAFE).read()
    for must in ("pub mod air_export;", "pub fn triton() -> Result<Self, GpuFault>",
                 "pub fn gpu_verifier() -> Option<&'static Verifier>", "pub fn gpu_node() -> Option<&'static GpuNode>",
                 "if device >= 32"):
        assert must in safe, must
    toml = open(os.path.join(ROOT, "neptune-core_amd", "rust", "neptune-hip", "Cargo.toml")).read()
    assert 'triton-constraint-builder = "1.0.0"' in toml and 'triton-constraint-circuit = "1.0.0"' in toml
