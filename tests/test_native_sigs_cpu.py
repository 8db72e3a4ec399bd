"""The ctypes signatures in ops/native.py against the HDS_EXPORT definitions in csrc/kernels/*.hip: same
argument count and compatible kinds (pointer / 32-bit int / 64-bit int / float / stream), so a signature typo fails
here instead of as a TypeError (or a silently mis-passed argument) on the GPU."""
import glob
import os
import re

from hcache_deepspeed_amd.ops import native

KDIR = os.path.join(os.path.dirname(native.__file__), "..", "csrc", "kernels")


def _exports():
    out = {}
    for path in glob.glob(os.path.join(KDIR, "*.hip")):
        src = open(path).read()
        for m in re.finditer(r"HDS_EXPORT\s+[\w\s\*]+?\b(hds_\w+)\s*\(([^)]*)\)", src):
            out[m.group(1)] = [a.strip() for a in m.group(2).replace("\n", " ").split(",") if a.strip()]
    return out


def _kind(decl):
    d = re.sub(r"\s+", " ", decl)
    if "*" in d or d.startswith("hipStream_t"):
        return "ps"
    if re.match(r"(const )?(int64_t|long|size_t)\b", d):
        return "l"
    if re.match(r"(const )?float\b", d):
        return "f"
    if re.match(r"(const )?(uint32_t|unsigned)\b", d):
        return "u"
    if re.match(r"(const )?(int|bool)\b", d):
        return "i"
    return "?"


def test_kernel_signatures_match_exports():
    ex = _exports()
    bad = []
    for name, spec in native._KERNEL_SIGS.items():
        if name not in ex:
            bad.append(f"{name}: no HDS_EXPORT definition")
            continue
        args = ex[name]
        if len(args) != len(spec):
            bad.append(f"{name}: {len(spec)} ctypes args vs {len(args)} in the source")
            continue
        for i, (c, a) in enumerate(zip(spec, args)):
            k = _kind(a)
            ok = (c in "ps" and k == "ps") or (c == k) or (c == "i" and k == "u")
            if not ok:
                bad.append(f"{name} arg {i}: '{c}' vs `{a}`")
    assert not bad, "\n".join(bad)


def test_host_signatures_match_exports():
    from hcache_deepspeed_amd.ops import host_sigs
    hdir = os.path.join(os.path.dirname(native.__file__), "..", "csrc", "host")
    ex = {}
    for path in glob.glob(os.path.join(hdir, "*.cpp")):
        src = open(path).read()
        for m in re.finditer(r"(?:HDS_EXPORT|HDS_HOST_EXPORT|extern \"C\")\s+[\w\s\*]+?\b(hds_\w+)\s*\(([^)]*)\)", src):
            ex[m.group(1)] = [a.strip() for a in m.group(2).replace("\n", " ").split(",")
                              if a.strip() and a.strip() != "void"]
    bad = [f"{n}: {len(a)} ctypes args vs {len(ex[n])} in the source" for n, (_, a) in host_sigs.SIGS.items()
           if n in ex and len(a) != len(ex[n])]
    missing = [n for n in host_sigs.SIGS if n not in ex]
    assert not bad and not missing, (bad, missing)


def test_shipped_fa_variants_only(monkeypatch):
    """HDS_ATTN_FWD_VAR may name only a forward variant the shipped library carries (2, 5, 20): a diagnostic or
    experiment variant raises instead of selecting a wrong-result kernel; the A/B library accepts it."""
    import pytest
    from hcache_deepspeed_amd.ops import build
    monkeypatch.delenv("HDS_KERNEL_LIB", raising=False)
    for v in ("2", "5", "20"):
        monkeypatch.setenv("HDS_ATTN_FWD_VAR", v)
        assert native.fwd_variant_default() == int(v)
    for v in ("13", "12", "11", "4"):
        monkeypatch.setenv("HDS_ATTN_FWD_VAR", v)
        with pytest.raises(ValueError, match="shipped FlashAttention library"):
            native.fwd_variant_default()
    monkeypatch.setenv("HDS_KERNEL_LIB", build.DIAG_LIB)
    monkeypatch.setenv("HDS_ATTN_FWD_VAR", "13")
    assert native.fwd_variant_default() == 13
    src = open(os.path.join(os.path.dirname(native.__file__), "..", "csrc", "kernels", "flash_attn_w64.hip")).read()
    # the shipped launcher instantiates only the default schedule outside the HDS_FA_DIAG block
    launch = src[src.index("int hds_attn_fwd_w64_launch"):]
    shipped = launch[:launch.index("#if HDS_FA_DIAG")]
    assert "attn_fwd_w64_kernel<128, 11>" in shipped and shipped.count("attn_fwd_w64_kernel<") == 1
