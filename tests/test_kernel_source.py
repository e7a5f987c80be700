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
