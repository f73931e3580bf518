"""INTEGRATION.md's Rust binding checked mechanically
against the C ABI it binds (include/onc_rpc.h): no Rust toolchain exists in
this image, so the `extern "C"` block cannot be compiled here, but every
function the header declares must be bound with the same parameters in the
same order and matching types, and every `#[repr(C)]` struct must list the
header's fields in the header's order with matching types."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

C_BASE = {"uint8_t": "u8", "uint32_t": "u32", "uint64_t": "u64", "int32_t": "i32", "int": "c_int",
          "double": "f64", "void": "c_void", "char": "c_char"}


def _strip_c_comments(s):
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def _c_type(t):
    """'const onc_batch*' -> '*const onc_batch'; 'uint64_t' -> 'u64'."""
    t = " ".join(t.replace("*", " * ").split())
    depth = t.count("*")
    toks = [x for x in t.split() if x != "*"]
    const = "const" in toks
    base = [x for x in toks if x != "const"][0]
    r = C_BASE.get(base, base)
    for d in range(depth):
        # only the innermost pointer carries the pointee's const
        r = ("*const " if (const and d == 0) else "*mut ") + r
    return r


def _header():
    s = _strip_c_comments(open(os.path.join(ROOT, "include", "onc_rpc.h")).read())
    funcs = {}
    for m in re.finditer(r"^([A-Za-z_][\w \*]*?)\b(onc_\w+)\s*\(([^;{]*?)\)\s*;", s, flags=re.M):
        ret, name, params = m.group(1).strip(), m.group(2), " ".join(m.group(3).split())
        ps = []
        if params and params != "void":
            for p in params.split(","):
                p = p.strip()
                pm = re.match(r"(.*?)(\w+)$", p)
                ps.append((pm.group(2), _c_type(pm.group(1))))
        funcs[name] = (_c_type(ret), ps)
    structs = {}
    for m in re.finditer(r"typedef struct (onc_\w+) \{(.*?)\} \1;", s, flags=re.S):
        body = m.group(2)
        if "union" in body:
            continue
        fields = []
        for line in body.split(";"):
            line = " ".join(line.split())
            if not line:
                continue
            fm = re.match(r"(.*?)(\w+)(\[(\d+)\])?$", line)
            ty = _c_type(fm.group(1))
            if fm.group(4):
                ty = f"[{ty}; {fm.group(4)}]"
            fields.append((fm.group(2), ty))
        structs[m.group(1)] = fields
    return funcs, structs


def _rust():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    code = "\n".join(re.findall(r"```rust\n(.*?)```", text, flags=re.S))
    code = re.sub(r"//[^\n]*", " ", code)
    funcs = {}
    for blk in re.findall(r'extern "C" \{(.*?)\n\}', code, flags=re.S):
        for m in re.finditer(r"pub fn (\w+)\((.*?)\)\s*(->\s*([^;]+))?;", blk, flags=re.S):
            params = " ".join(m.group(2).split())
            ps = []
            if params:
                for p in params.split(","):
                    n, t = p.split(":", 1)
                    ps.append((n.strip(), " ".join(t.split())))
            funcs[m.group(1)] = ((m.group(4) or "()").strip(), ps)
    structs = {}
    for m in re.finditer(r"pub struct (onc_\w+) \{(.*?)\}", code, flags=re.S):
        fields = []
        for f in m.group(2).split(","):
            f = " ".join(f.split())
            if not f or not f.startswith("pub "):
                continue
            n, t = f[4:].split(":", 1)
            fields.append((n.strip().replace("r#", ""), " ".join(t.split())))
        structs[m.group(1)] = fields
    return funcs, structs


def test_every_header_function_is_bound_with_matching_signature():
    cf, _ = _header()
    rf, _ = _rust()
    assert len(cf) >= 20, sorted(cf)
    missing = sorted(set(cf) - set(rf))
    assert not missing, f"INTEGRATION.md does not bind {missing}"
    for name, (ret, params) in cf.items():
        rret, rparams = rf[name]
        assert rret == ret, (name, rret, ret)
        assert [t for _, t in rparams] == [t for _, t in params], (name, rparams, params)
    extra = sorted(n for n in rf if n.startswith("onc_") and n not in cf)
    assert not extra, f"bound but not in the header: {extra}"


@pytest.mark.parametrize("name", ["onc_auth", "onc_unix_params", "onc_batch", "onc_decoded", "onc_iov_rec"])
def test_repr_c_structs_match_header(name):
    _, cs = _header()
    _, rs = _rust()
    assert name in cs and name in rs
    assert rs[name] == cs[name], (rs[name], cs[name])
