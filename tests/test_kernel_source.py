"""Source checks on the product kernels (CPU suite).

Round 4's faulting A/B build widened ``__builtin_amdgcn_readfirstlane``'s
``int`` result straight into a 64-bit address, which sign-extends from 2^31
(DESIGN_LOG.md 1.8).  The kernels now read lanes only through ``rfl_u32`` /
``rl_u32``, which return ``uint32_t``; this test keeps it that way."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "zeroskip_amd", "csrc")


def _product_sources():
    for name in sorted(os.listdir(CSRC)):
        if name.endswith((".hip", ".cpp", ".h", ".c")):
            yield name, open(os.path.join(CSRC, name)).read()


def test_lane_reads_only_in_the_u32_helpers():
    for name, src in _product_sources():
        for m in re.finditer(r"__builtin_amdgcn_read(first)?lane\s*\(", src):
            # the enclosing function: the last definition line before the use
            head = src[:m.start()]
            fn = re.findall(r"__device__ __forceinline__ (\w+) (\w+)\(", head)
            assert fn and fn[-1] in (("uint32_t", "rfl_u32"), ("uint32_t", "rl_u32")), \
                f"{name}: lane read outside rfl_u32/rl_u32 at offset {m.start()}: {src[m.start():m.start() + 80]!r}"
            # and that helper's body is one return with a uint32_t cast
            body = src[head.rfind("{"):src.index("}", m.start())]
            assert "return (uint32_t)__builtin_amdgcn_read" in body, name


def test_no_signed_lane_read_widened():
    """No helper result is cast to a signed 64-bit type (that would
    sign-extend again)."""
    for name, src in _product_sources():
        assert not re.search(r"\((int64_t|long|long long|intptr_t|ptrdiff_t)\)\s*r(fl|l)_u32", src), name


# Every list the kernels fill through an atomic slot counter and cut at a cap
# (VERDICT r05 next #2).  Which entries such a list holds past its cap depends
# on the order the waves found them, so every consumer must be order-
# independent: it uses the list only when the count fits the cap, and then
# compares it as a sorted / set-valued whole, or it falls back to a full pass.
# The table names each site's enclosing function and that consumer rule
# ("Capped lists"); a new capped list fails this test until it
# is reviewed and added here.
CAPPED_LISTS = {
    # commit verdict (zscrc_device_verify_commits_verdict*): count exact,
    # indices "in no particular order" (include/zscrc.h); libzscrc's files
    # path sorts them when nbad <= cap and re-verifies every commit's status
    # otherwise (zscrc_files.cpp); cpass classifies min(nbad, cap) entries
    # and reports complete = 0 past LIST_CAP; tests compare sets.
    "emit": "verdict",
    "part_fold_kernel": "verdict",        # long commits: the verdict after the part fold
    # out-of-image commits listed by the classify passes into the same verdict
    "classify_scatter": "verdict",
    "classify_only3": "verdict",
    # the one-launch class-3 verdict (xteam_kernel MODE 3): out-of-image
    # commits listed by workgroup 0's scan, the rest by nbv_check (MODE 3 or its fold)
    "xteam_kernel": "verdict",
    "nbv_check": "verdict",
    # cpass post kernel: the first out_cap classified entries go to the host
    # block; counts (nbad, nstale) are over every classified entry, published
    # by the last workgroup; the host and the device row read the same block
    "cpass_post_kernel": "cpass block",
    # consistent.py mismatch_rows: rows used only when count <= ROWS_CAP
    # (None -> the host path), then sorted by commit index
    "mismatch_rows_kernel": "rows",
}


def _enclosing_function(src: str, at: int) -> str:
    head = src[:at]
    names = re.findall(r"(?:__global__|__device__)[^\n]*?\b(?!__launch_bounds__)(\w+)\s*\(", head)
    return names[-1] if names else "?"


def test_capped_lists_are_reviewed():
    src = open(os.path.join(CSRC, "zscrc_kernels.hip")).read()
    sites = {}
    for m in re.finditer(r"if \((k|slot) (<|>=) [\w.]*cap\)", src):
        fn = _enclosing_function(src, m.start())
        sites[fn] = sites.get(fn, 0) + 1
    unknown = sorted(set(sites) - set(CAPPED_LISTS))
    assert not unknown, f"capped list in {unknown}: review its consumers (DESIGN.md §7) and add it here"
    assert sites, "no capped list found: the pattern no longer matches the kernels"
