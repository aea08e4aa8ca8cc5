"""CPU tests of the C ABI boundary: the library loads, exports every symbol the
public headers declare, and the host-side checks/dispatch logic behave -- no
kernel is launched (no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INCLUDE = os.path.join(ROOT, "include")


def _fa():
    import fa_mi355x

    return fa_mi355x


def _declared_functions(header):
    text = open(os.path.join(INCLUDE, header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"//.*", "", text)
    # return-type name(  ... ) ;   at file scope (no typedef/struct bodies)
    names = re.findall(r"^[A-Za-z_][\w \*]*?\b([a-z_][a-z0-9_]*)\s*\([^;{]*\)\s*;", text, re.M)
    return sorted(set(names))


def _dynsyms():
    lib = _fa().library_path()
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True,
                         check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_library_loads():
    fa = _fa()
    assert os.path.exists(fa.library_path())
    assert "gfx950" in fa.version()


def test_exports_every_c_abi_symbol():
    declared = _declared_functions("fa_mi355x.h")
    assert "fa_fwd_f16" in declared and len(declared) >= 10
    syms = _dynsyms()
    missing = [d for d in declared if d not in syms]
    assert not missing, f"declared but not exported: {missing}"
    assert set(declared) == set(_fa().EXPORTED_SYMBOLS)


def test_exports_reference_cpp_signature():
    declared = _declared_functions("flash_attention_v9.h")
    assert declared == ["flash_attention_v9_dispatch"]
    lib = _fa().library_path()
    out = subprocess.run(["nm", "-DC", "--defined-only", lib], capture_output=True, text=True,
                         check=True).stdout
    assert re.search(r"flash_attention_v9_dispatch\(__half const\*, __half const\*, __half const\*,"
                     r" __half\*, float\*, float\*, int, int, int, int, bool, ihipStream_t\*\)",
                     out), out


KVPAIR_LDS = 4 * 64 * 256 + 4 * 8 * 64 * 16  # tile buffers + shared Q (csrc kKvpairLdsBytes)


def test_config_table():
    fa = _fa()
    cfgs = fa.configs()
    assert [c.id for c in cfgs] == list(range(len(cfgs)))
    for c in cfgs:
        assert c.head_dim in (64, 128) and c.dtype in ("float16", "bfloat16")
        assert c.block_n % 32 == 0
        if "_kvpair_" in c.name:
            # two waves per 32 query rows; LDS = 4 tile buffers + the shared
            # Q of 4 row sets (8 KB each), which also covers the merge region
            assert c.block_m == 16 * c.waves
            assert c.lds_bytes == KVPAIR_LDS >= 4 * 17 * 64 * 16
            continue
        if "_kvquad_" in c.name:
            # four waves per 32 query rows; four double-width stage buffers
            assert c.block_m == 8 * c.waves
            assert c.lds_bytes == 4 * 2 * c.block_n * 256
            continue
        # 64 query rows per wave (one wave per SIMD) or 32
        assert c.block_m == (64 if "_w4x64_" in c.name else 16 if "_w4x16_" in c.name else 32) * c.waves
        # K and V image buffers of 256-B row slots: double-buffered, or three
        # rotating buffers each for the LDS-DMA configs
        nbuf = 3 if "_dma_" in c.name else 2
        if any(t in c.name for t in ("_asm_persistent_", "_asm_pair_", "_asm_single_", "_asm_mixed_", "_asm_planned_")) and c.head_dim == 128:
            nbuf = 4  # the W4 / W4P pair programs' two key tiles per barrier (gen_w4*_item.py)
        need = 2 * nbuf * c.block_n * 256
        if "_pingpong_persistent_" in c.name and "_dma_" not in c.name and not c.causal:
            need = max(need, KVPAIR_LDS)  # room for the KV-pair tail halves
        if "_w4x64_" in c.name and "_asm_quad_" not in c.name:
            need += 256 * 64  # the item table (256 slots of 16 dwords)
        assert c.lds_bytes == need <= 160 * 1024
    # every (waves, bn) non-split config exists for both masks
    nonsplit = {(c.waves, c.block_n, c.causal) for c in cfgs if not c.split_kv}
    for w, bn, _ in list(nonsplit):
        assert (w, bn, True) in nonsplit and (w, bn, False) in nonsplit


@pytest.mark.parametrize("causal", [False, True])
def test_select_config(causal):
    fa = _fa()
    cfgs = fa.configs()
    for s in (1, 64, 512, 1024, 2048, 4096, 8192, 16384):
        for b, h in ((1, 32), (64, 32), (8, 32), (1, 1)):
            cid = fa.select_config(b, h, s, causal)
            c = cfgs[cid]
            assert c.causal == causal and not c.split_kv
    # B=1 H=32 S=1024 (BASELINE config 1): the paired tier (one round of
    # pairs); the long launches: the persistent tier
    assert "_asm_pair_" in cfgs[fa.select_config(1, 32, 1024, causal)].name
    assert "_persistent_" in cfgs[fa.select_config(1, 32, 8192, causal)].name
    # causal launches of <= 2 rounds of pairs up to S=2048: the paired tier;
    # non-causal ones of <= 256 64-row blocks under 3/4 of a round: the KV-quad
    # launches of <= 1 64-row block per CU (heads of <= 64 blocks): one block
    # per workgroup on the paired tier's program
    for b, h, s in ((1, 8, 2048), (1, 32, 512), (1, 32, 256), (1, 4, 4096), (1, 64, 256), (1, 32, 128),
                    (4, 32, 128), (1, 1, 1)):
        assert "_asm_single_" in cfgs[fa.select_config(b, h, s, causal)].name, (b, h, s, causal)
    assert "_w4_" in cfgs[fa.select_config(16, 32, 128, causal)].name
    # S <= 256 past one block per CU: one round of pairs (causal: or mixed)
    assert "_asm_pair_" in cfgs[fa.select_config(1, 96, 256, causal)].name
    assert "_asm_pair_" in cfgs[fa.select_config(1, 200, 128, causal)].name
    assert "_asm_single_" not in cfgs[fa.select_config(1, 4, 8192, causal)].name  # 128 blocks per head
    assert "_asm_pair_" in cfgs[fa.select_config(1, 16, 2048, causal)].name  # 512 blocks
    # between the KV-quad's and the paired tier's non-causal shapes over long
    # heads: the KV-pair; shorter heads: one round of pairs
    assert "_asm_pair_" in cfgs[fa.select_config(1, 20, 1024, False)].name
    assert "_kvpair_" in cfgs[fa.select_config(1, 5, 4160, False)].name  # long heads (65 blocks)
    # long heads, few of them: causal -> the KV-quad's four-way key split
    # (the _ws entries run the split tier there), non-causal -> the paired tier
    want = "_kvquad_" if causal else "_asm_pair_"
    for b, h, s in ((1, 4, 8192), (1, 2, 16384)):
        assert want in cfgs[fa.select_config(b, h, s, causal)].name, (b, h, s, causal)
    for b, h, s in ((1, 16, 2048), (1, 8, 4096), (2, 8, 2048)):  # <= 1 round of pairs
        assert "_asm_pair_" in cfgs[fa.select_config(b, h, s, causal)].name, (b, h, s, causal)
    if causal:  # one to two blocks per CU: the heaviest blocks alone, the rest paired
        for b, h, s in ((1, 32, 768), (1, 24, 1024), (3, 8, 1024), (1, 12, 2048)):
            assert "_asm_mixed_" in cfgs[fa.select_config(b, h, s, True)].name, (b, h, s)
    if causal:  # 2-4 blocks per CU short of whole quads: groups planned on the host
        for b, h, s in ((1, 32, 1280), (1, 32, 1536), (1, 16, 2560), (1, 25, 2048)):
            assert "_asm_planned_" in cfgs[fa.select_config(b, h, s, True)].name, (b, h, s)
    if causal:  # 1-2 rounds of pairs: two pairs per workgroup
        for b, h, s in ((1, 32, 2048), (2, 32, 1024), (1, 16, 4096)):
            assert "_asm_quad_" in cfgs[fa.select_config(b, h, s, True)].name, (b, h, s)


def _null_call(lib, head_dim=128, b=1, h=1, s=64, causal=0, ptr=None):
    p = ctypes.c_void_p(ptr)
    return lib.fa_fwd_f16(p, p, p, p, b, h, s, head_dim, causal, None)


def test_argument_errors_without_gpu():
    fa = _fa()
    lib = fa.load_library()
    assert _null_call(lib, head_dim=96) == fa.FA_ERR_UNSUPPORTED_HEAD_DIM
    assert _null_call(lib, head_dim=256) == fa.FA_ERR_UNSUPPORTED_HEAD_DIM
    assert _null_call(lib, head_dim=64) == fa.FA_ERR_NULL_POINTER  # 64 is supported
    assert _null_call(lib, b=-1) == fa.FA_ERR_BAD_SHAPE
    assert _null_call(lib, s=-5) == fa.FA_ERR_BAD_SHAPE
    assert _null_call(lib) == fa.FA_ERR_NULL_POINTER
    # a head's byte range must fit the 32-bit buffer resource
    assert _null_call(lib, s=(1 << 23) - 1) == fa.FA_ERR_NULL_POINTER
    assert _null_call(lib, s=1 << 23) == fa.FA_ERR_BAD_SHAPE
    assert _null_call(lib, s=1 << 23, head_dim=64) == fa.FA_ERR_NULL_POINTER
    assert _null_call(lib, b=0) == fa.FA_OK  # empty problem: nothing to launch
    assert _null_call(lib, s=0) == fa.FA_OK
    assert _null_call(lib, b=1 << 16, h=1 << 16) == fa.FA_ERR_BAD_SHAPE
    p = ctypes.c_void_p(None)
    q = ctypes.c_void_p(0x1000)  # never dereferenced: every call below fails validation
    assert lib.fa_fwd_f16_config(q, q, q, q, 1, 1, 64, 128, 0, 999, None) == fa.FA_ERR_BAD_CONFIG
    # config 0 is non-causal: asking it for causal is rejected before any launch
    assert lib.fa_fwd_f16_config(q, q, q, q, 1, 1, 64, 128, 1, 0, None) == fa.FA_ERR_BAD_CONFIG
    assert lib.fa_fwd_f16_splitkv(p, p, p, p, 1, 1, 64, 64, 0, 0, p, p, None) == \
        fa.FA_ERR_UNSUPPORTED_HEAD_DIM
    assert lib.fa_fwd_f16_splitkv(q, q, q, q, 1, 1, 64, 128, 0, 2, p, p, None) == \
        fa.FA_ERR_WORKSPACE
    assert lib.fa_fwd_f16_splitkv(q, q, q, q, 1, 1, 64, 128, 0, 65, q, q, None) == \
        fa.FA_ERR_BAD_CONFIG
    # fp32 partial rows: half the main path's sequence range
    assert lib.fa_fwd_f16_splitkv(q, q, q, q, 1, 1, 1 << 22, 128, 0, 2, q, q, None) == \
        fa.FA_ERR_BAD_SHAPE


def test_status_strings():
    lib = _fa().load_library()
    for st in range(8):
        assert lib.fa_status_string(st).decode() not in ("", "unknown status")
    assert lib.fa_status_string(99).decode() == "unknown status"


def test_splitkv_sizes():
    lib = _fa().load_library()
    assert lib.fa_splitkv_o_bytes(2, 3, 100, 128, 4) == 4 * 2 * 3 * 100 * 128 * 4
    assert lib.fa_splitkv_ml_bytes(2, 3, 100, 128, 4) == 4 * 2 * 3 * 100 * 2 * 4
    assert lib.fa_splitkv_o_bytes(0, 3, 100, 128, 4) == 0
    for s in (1, 64, 1000, 8192):
        n = lib.fa_splitkv_num_splits(1, 4, s, 1)
        assert 1 <= n <= 16 and n <= (s + 63) // 64


def test_kernel_attrs_needs_runtime():
    """fa_kernel_attrs reads compiled metadata through the HIP runtime; without a
    GPU it must fail cleanly (status), never crash."""
    fa = _fa()
    try:
        import torch

        has_gpu = torch.cuda.is_available()
    except ImportError:
        has_gpu = False
    if has_gpu:
        pytest.skip("GPU present: covered by the gpu tests")
    with pytest.raises(fa.FlashAttentionError):
        fa.kernel_attrs(0)


def test_python_mirror_rejects_bad_tensors():
    torch = pytest.importorskip("torch")
    fa = _fa()
    x = torch.zeros(1, 1, 8, 128, dtype=torch.float32)
    with pytest.raises(fa.FlashAttentionError):
        fa.flash_attention_fwd(x, x, x)
    y = torch.zeros(1, 1, 8, 128, dtype=torch.float16)  # host tensor
    with pytest.raises(fa.FlashAttentionError):
        fa.flash_attention_fwd(y, y, y)


def test_fp16_only_entries_reject_bf16():
    """The split-KV entry and the reference-signature mirror are fp16-only
    (the reference's half* boundary, flash_attention.cu:606-611): bf16 tensors
    raise before any pointer reaches the library (checked without a GPU)."""
    torch = pytest.importorskip("torch")
    fa = _fa()
    x = torch.zeros(1, 1, 8, 128, dtype=torch.bfloat16)
    with pytest.raises(fa.FlashAttentionError, match="float16"):
        fa.flash_attention_fwd_splitkv(x, x, x, causal=False)
    with pytest.raises(fa.FlashAttentionError, match="float16"):
        fa.flash_attention_v9_dispatch(x, x, x, x, None, None, 1, 1, 8, 128, False)
    y = torch.zeros(1, 1, 8, 128, dtype=torch.float32)
    with pytest.raises(fa.FlashAttentionError, match="float16"):
        fa.flash_attention_v9_dispatch(y, y, y, y, None, None, 1, 1, 8, 128, True)


TWIN_PREFIXES = ("", "bf16_", "d64_", "bf16_d64_")


def test_config_table_ships_only_used_tiers():
    """Every shipped config is a tier the dispatcher picks (or a dtype /
    head_dim twin of one), the explicit split-KV entry, or a baseline a test
    compares against -- no dead experiments in the library."""
    fa = _fa()
    cfgs = fa.configs()
    by_name = {c.name: c for c in cfgs}
    used = set()
    for causal in (False, True):
        for s in (1, 64, 128, 200, 256, 300, 512, 768, 1024, 2048, 4096, 4160, 8192, 16384, 32768):
            for b, h in ((1, 1), (1, 2), (1, 4), (1, 5), (1, 8), (1, 16), (1, 32), (1, 64), (2, 32),
                         (4, 32), (8, 32), (16, 32), (64, 32), (3, 40), (1, 203), (1, 20)):
                base = cfgs[fa.select_config(b, h, s, causal)].name
                used |= {pre + base for pre in TWIN_PREFIXES if pre + base in by_name}
    baselines = {"bm256_bn64_w8_m16_pingpong_noncausal", "bm256_bn64_w8_m16_pingpong_causal",
                 "bm256_bn64_w8_m16_pingpong_persistent_dma_noncausal",
                 "bm256_bn64_w8_m16_pingpong_persistent_dma_causal",
                 # the W4 kernel's same-arithmetic baselines (test_w4_gpu.py), and
                 # the anchor the head_dim-64 fallback twins are looked up from
                 "bm256_bn64_w8_m16_pingpong_persistent_causal",
                 "bf16_bm256_bn64_w8_m16_pingpong_persistent_causal",
                 "bm256_bn64_w8_m16_pingpong_persistent_noncausal",
                 "bf16_bm256_bn64_w8_m16_pingpong_persistent_noncausal"}
    explicit = {c.name for c in cfgs if c.split_kv}
    # BN=128 (the reference's long non-causal tile, flash_attention.cu:626-634):
    # built, parity-tested and measured, not dispatched (BN=128)
    explicit |= {c.name for c in cfgs if c.block_n == 128}
    # the quad grouping without a mask: parity-tested, slower than the
    # persistent tier wherever it could run (profiles/r05_w4q_ab.jsonl)
    explicit |= {c.name for c in cfgs if "_asm_quad_noncausal" in c.name}
    # head_dim 64 of the asm W4 tier runs the ping-pong persistent twins
    w4 = {n for n in used if "_asm_persistent_" in n}
    assert w4, "the W4 tier is dispatched"
    used |= {pre + "bm256_bn64_w8_m16_pingpong_persistent_" + ("causal" if n.endswith("_causal")
                                                                else "noncausal")
             for n in w4 for pre in ("d64_", "bf16_d64_")}
    unused = sorted(set(by_name) - used - baselines - explicit)
    assert not unused, unused
    # every dispatched fp16 d128 tier has all three twins (W4: the bf16 one)
    for name in used:
        if not name.startswith(("bf16_", "d64_")):
            pres = ("bf16_",) if "_asm_" in name else TWIN_PREFIXES  # W4 / W4P: bf16 only
            assert all(pre + name in by_name for pre in pres), name


def test_bf16_configs_and_entry_points():
    """bf16 twins exist for the dispatched tiers; each entry point accepts
    only its own dtype's configs (checked before any launch: no GPU needed)."""
    fa = _fa()
    lib = fa.load_library()
    cfgs = fa.configs()
    bf = [c for c in cfgs if c.dtype == "bfloat16"]
    assert {c.causal for c in bf} == {False, True}
    assert all(not c.split_kv for c in bf)
    p = ctypes.c_void_p(0x1000)
    f16_id = next(c.id for c in cfgs if c.dtype == "float16" and not c.causal and not c.split_kv)
    bf_id = next(c.id for c in bf if not c.causal)
    assert lib.fa_fwd_bf16_config(p, p, p, p, 1, 1, 64, 128, 0, f16_id, None) == fa.FA_ERR_BAD_CONFIG
    assert lib.fa_fwd_f16_config(p, p, p, p, 1, 1, 64, 128, 0, bf_id, None) == fa.FA_ERR_BAD_CONFIG
    assert lib.fa_fwd_bf16(p, p, p, p, 1, 1, 64, 96, 0, None) == fa.FA_ERR_UNSUPPORTED_HEAD_DIM
    # a forced config must match the call's head_dim
    d64 = next(c.id for c in cfgs if c.head_dim == 64 and c.dtype == "float16" and not c.causal)
    assert lib.fa_fwd_f16_config(p, p, p, p, 1, 1, 64, 128, 0, d64, None) == \
        fa.FA_ERR_UNSUPPORTED_HEAD_DIM
    # the dispatcher's tier for each shape has a bf16 twin
    for s in (64, 1024, 4096):
        for b, h in ((1, 32), (64, 32)):
            for causal in (False, True):
                c = cfgs[fa.select_config(b, h, s, causal)]
                assert any(t.waves == c.waves and t.causal == c.causal and t.block_m == c.block_m
                           for t in bf), c.name


def test_split_plan_and_workspace_entry():
    """The causal split tier's plan (fa_fwd_split_pieces / fa_fwd_ws_bytes)
    and the workspace entry's argument checks -- no launch, no GPU needed."""
    fa = _fa()
    lib = fa.load_library()
    # the dispatcher splits long causal launches short of the persistent tier
    for b, h, s in ((1, 6, 8192), (1, 4, 8192), (1, 2, 16384), (1, 1, 32768)):
        t = lib.fa_fwd_split_pieces(b, h, s, 128, 1)
        assert t >= 4, (b, h, s)
        need = lib.fa_fwd_ws_bytes(b, h, s, 128, 1, 0)
        assert need > 0 and need % 256 == 0
    # no split: non-causal, head_dim 64, the persistent tier's shapes, S < 4096
    # and the paired tier's shapes (B=1 H<=8 S=4096)
    for args in ((1, 4, 4096, 128, 0), (1, 4, 4096, 64, 1), (64, 32, 4096, 128, 1),
                 (1, 32, 8192, 128, 1), (1, 32, 1024, 128, 1), (1, 8, 2048, 128, 1),
                 (1, 8, 4096, 128, 1), (1, 4, 4096, 128, 1)):
        assert lib.fa_fwd_split_pieces(*args) == 0, args
        # the W4 tier's cross-XCD tail pool wants the 64-KB counter region on
        # launches of >= 16 rounds in the snake order (the headline); none
        # on the causal pairs' shapes (<= 64 heads) or other tiers
        want = 65536 if args in ((64, 32, 4096, 128, 1),) else 0
        assert lib.fa_fwd_ws_bytes(*args, 0) == want, args
    # a forced piece length: sizes grow with the pieces per block; > 8 pieces,
    # non-causal or one piece per block is not a split
    assert lib.fa_fwd_ws_bytes(1, 32, 1024, 128, 1, 6) > 0
    assert lib.fa_fwd_ws_bytes(1, 32, 1024, 128, 1, 1) == 0   # 16 pieces
    assert lib.fa_fwd_ws_bytes(1, 32, 1024, 128, 0, 6) == 0
    assert lib.fa_fwd_ws_bytes(1, 32, 1024, 128, 1, 16) == 0  # one piece
    need = lib.fa_fwd_ws_bytes(1, 4, 8192, 128, 1, 0)
    p = ctypes.c_void_p(0x1000)
    assert lib.fa_fwd_f16_ws(p, p, p, p, 1, 4, 8192, 128, 1, 0, None, need, None) == fa.FA_ERR_WORKSPACE
    assert lib.fa_fwd_f16_ws(p, p, p, p, 1, 4, 8192, 128, 1, 0, p, need - 1, None) == fa.FA_ERR_WORKSPACE
    assert lib.fa_fwd_f16_ws(p, p, p, p, 1, 32, 1024, 128, 1, 1, p, 1 << 30, None) == fa.FA_ERR_BAD_CONFIG
    assert lib.fa_fwd_bf16_ws(p, p, p, p, 1, 4, 8192, 96, 1, 0, p, need, None) == \
        fa.FA_ERR_UNSUPPORTED_HEAD_DIM
    assert lib.fa_fwd_f16_ws(None, p, p, p, 1, 4, 8192, 128, 1, 0, p, need, None) == fa.FA_ERR_NULL_POINTER


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc")
def test_no_kernel_uses_scratch():
    """Compile-time twin of test_fullsize_gpu.test_register_report: every
    kernel of the library -- the asm item programs included, whose statement
    leaves hipcc 20 VGPRs for whatever is live across it -- keeps all of its
    state in registers (ScratchSize 0), checked from hipcc's resource-usage
    remarks so a spill is caught without a GPU."""
    pkg = os.path.join(ROOT, "flash-attention-cuda_amd")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-fno-honor-nans",
           "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(pkg, "csrc"), "-c",
           os.path.join(pkg, "csrc", "fa_fwd.hip"), "-o", os.devnull,
           "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    names = re.findall(r"Function Name: (\S+)", out.stderr)
    scratch = [int(x) for x in re.findall(r"ScratchSize \[bytes/lane\]: (\d+)", out.stderr)]
    assert names and len(names) == len(scratch), (len(names), len(scratch))
    spills = {n: s for n, s in zip(names, scratch) if s}
    assert not spills, spills


def test_generated_item_program_is_current(tmp_path):
    """The committed asm item program (csrc/fa_w4_item.inc) is exactly what
    csrc/gen_w4_item.py generates: the Makefile regenerates it by mtime only,
    so after a checkout a stale include could otherwise be compiled."""
    import sys

    csrc = os.path.join(ROOT, "flash-attention-cuda_amd", "csrc")
    out = tmp_path / "fa_w4_item.inc"
    env = {k: v for k, v in os.environ.items() if not k.startswith("W4_")}  # no experiment knobs
    subprocess.run([sys.executable, os.path.join(csrc, "gen_w4_item.py"), str(out)], check=True,
                   env=env, timeout=300)
    with open(os.path.join(csrc, "fa_w4_item.inc")) as f:
        committed = f.read()
    assert out.read_text() == committed, "fa_w4_item.inc is stale: run `make -C flash-attention-cuda_amd`"


def test_generated_pair_program_is_current(tmp_path):
    """The committed paired-tier program (csrc/fa_w4p_item.inc) is exactly what
    csrc/gen_w4p_item.py generates, and its stamps variant generates."""
    import sys

    csrc = os.path.join(ROOT, "flash-attention-cuda_amd", "csrc")
    env = {k: v for k, v in os.environ.items() if not k.startswith("W4")}
    out = tmp_path / "fa_w4p_item.inc"
    subprocess.run([sys.executable, os.path.join(csrc, "gen_w4p_item.py"), str(out)], check=True,
                   env=env, timeout=300)
    with open(os.path.join(csrc, "fa_w4p_item.inc")) as f:
        assert out.read_text() == f.read(), "fa_w4p_item.inc is stale: run `make -C flash-attention-cuda_amd`"
    env["W4P_DIAG"] = "stamps"
    subprocess.run([sys.executable, os.path.join(csrc, "gen_w4p_item.py"), str(out)], check=True,
                   env=env, timeout=300)
    text = out.read_text()
    for fn in ("w4p_item_causal_f16", "w4p_item_noncausal_bf16"):
        assert f"void {fn}(" in text, fn
    assert "s_memtime" in text


@pytest.mark.parametrize("env", [
    {"W4_XP": "rsa"}, {"W4_XP": "cvtearly"}, {"W4_XP": "kpre"}, {"W4_XP": "shift4"},
    {"W4_XP": "nomfz"}, {"W4_XP": "twobar"}, {"W4_WAGE": "0"}, {"W4_V_AHEAD": "5"}, {"W4_DIAG": "stamps"},
    {"W4_DIAG": "prostamps"}, {"W4_XP": "mix"}, {"W4_XP": "noepi,noqscale,nofirst"}, {"W4_XP": "epinostore"}, {"W4_XP": "p1dmaa"},
], ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()))
def test_generator_variants_generate(tmp_path, env):
    """The experiment / diagnostic switches DESIGN.md cites (tools/w4_variant.sh
    builds) still generate a complete item program: every filler lands in an
    MFMA gap and every function is emitted."""
    import sys

    csrc = os.path.join(ROOT, "flash-attention-cuda_amd", "csrc")
    out = tmp_path / "fa_w4_item.inc"
    e = {k: v for k, v in os.environ.items() if not k.startswith("W4_")}
    e.update(env)
    subprocess.run([sys.executable, os.path.join(csrc, "gen_w4_item.py"), str(out)], check=True,
                   env=e, timeout=300)
    text = out.read_text()
    for fn in ("w4_item_noncausal_f16", "w4_item_causal_bf16", "w4_item_causal_split_f16",
               "w4_item_causal_d64_f16"):
        assert f"void {fn}(" in text, fn


def test_tail_pool_workspace_sizing():
    """fa_fwd_ws_bytes asks for the 64-KB counter region exactly where the W4
    tier runs its cross-XCD tail pool: >= 64 rounds of 256-row items per XCD
    in the snake order (256 CUs: >= 2048 items per XCD), never on the causal
    pairs (<= 64 heads) or other tiers -- no launch, no GPU needed."""
    lib = _fa().load_library()
    pool = [(64, 32, 4096, 128, 1), (32, 32, 4096, 128, 1), (16, 32, 8192, 128, 0),
            (64, 32, 4096, 64, 1), (128, 24, 2048, 128, 1)]
    none = [(16, 32, 4096, 128, 1),   # 32 rounds
            (1, 32, 8192, 128, 1),    # causal pairs
            (1, 32, 16384, 128, 1),
            (8, 32, 4096, 128, 1),    # 16 rounds
            (1, 32, 1024, 128, 1),    # the paired short tier
            (64, 32, 4096, 96, 1)]    # unsupported head_dim
    for args in pool:
        assert lib.fa_fwd_ws_bytes(*args, 0) == 65536, args
        assert lib.fa_fwd_split_pieces(*args) == 0, args
    for args in none:
        assert lib.fa_fwd_ws_bytes(*args, 0) == 0, args
