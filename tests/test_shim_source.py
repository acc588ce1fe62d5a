"""CPU: static checks of the cgo shim's source (no Go toolchain in this image).

- `&s[0]` of an empty Go slice panics, and the ABI takes NULL with a zero count for every
  array: the only `&x[0]` left is inside `ptr`, the helper every slice goes through.
- Every `C.esc_*` the shim calls is declared in include/escalator_hip.h.
"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "go", "escalatorhip", "escalatorhip.go")


def _code(path):
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)            # block comments (the cgo preamble too)
    return "\n".join(line.split("//", 1)[0] for line in src.splitlines())


def test_no_unguarded_first_element_address():
    code = _code(SHIM)
    hits = [m.start() for m in re.finditer(r"&\s*\w+(\.\w+)*\s*\[\s*0\s*\]", code)]
    body = re.search(r"func ptr\[T any\]\(s \[\]T\) \*T \{(.*?)\n\}", code, flags=re.S)
    assert body, "the ptr helper is missing"
    assert all(body.start(1) <= h < body.end(1) for h in hits), [code[h - 40:h + 20] for h in hits]
    assert "if len(s) == 0" in body.group(1)


def test_shim_calls_only_declared_abi():
    from escalator_amd import _lib as L
    declared = set(L.header_functions())
    called = set(re.findall(r"C\.(esc_[a-z_0-9]+)\s*\(", _code(SHIM)))
    assert called and called <= declared, sorted(called - declared)
    assert "esc_ctx_create_multi" in called and "esc_ctx_counts" in called
