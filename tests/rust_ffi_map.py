"""C header -> Rust FFI mapping shared by scripts/gen_rust_ffi.py (writes rust/src/gpu/ffi.rs) and
tests/test_rust_shim.py (checks the committed file against include/crdt_gpu.h)."""
import re

_SCALAR = {
    "int": "c_int", "unsigned": "c_uint", "size_t": "usize", "uint64_t": "u64", "uint32_t": "u32",
    "uint8_t": "u8", "int8_t": "i8", "char": "c_char", "void": "c_void",
}
_RESERVED = {"self", "in", "type", "ref", "mut", "fn", "use", "loop", "move", "box", "match", "where"}


def _strip_comments(text: str) -> str:
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return re.sub(r"//[^\n]*", "", text)


def rust_type(ctype: str) -> str:
    """`const uint64_t *` -> `*const u64`, `crdt_ctx **` -> `*mut *mut crdt_ctx`, `int` -> `c_int`;
    a function pointer `int (*)(void *user, size_t n)` -> `Option<unsafe extern "C" fn(*mut c_void,
    usize) -> c_int>` (NULL-able, as the header allows)."""
    fm = re.match(r"^(.*?)\(\s*\*\s*\)\s*\((.*)\)$", " ".join(ctype.split()))
    if fm:
        ret, params = fm.group(1).strip(), fm.group(2).strip()
        args = [] if params in ("", "void") else [rust_type(_split_decl(p.strip())[0]) for p in params.split(",")]
        r = rust_type(ret)
        return 'Option<unsafe extern "C" fn(' + ", ".join(args) + ")" + ("" if r == "()" else " -> " + r) + ">"
    t = " ".join(ctype.replace("*", " * ").split())
    if t == "void":
        return "()"
    stars = t.count("*")
    base = t.replace("*", "").strip()
    const = base.startswith("const ")
    base = base.replace("const ", "").strip()
    rt = _SCALAR.get(base, base)
    for i in range(stars):
        rt = ("*const " if (const and i == 0) else "*mut ") + rt
    return rt


def rust_field(name: str) -> str:
    return name + "_" if name in _RESERVED else name


def rust_param(name: str, i: int) -> str:
    if not name:
        return f"arg{i}"
    return name + "_" if name in _RESERVED else name


def const_type(name: str) -> str:
    return "c_uint" if name == "CRDT_ACCUMULATE" else "c_int"


def _split_decl(decl: str):
    """'const uint64_t *in' -> ('const uint64_t *', 'in'); array params 'uint8_t *id' ok."""
    decl = " ".join(decl.split())
    m = re.match(r"^(.*?)([A-Za-z_][A-Za-z0-9_]*)$", decl)
    if not m:
        raise ValueError(decl)
    ctype, name = m.group(1).strip(), m.group(2)
    if not ctype:  # a bare type with no name
        return name, ""
    return ctype, name


def parse_header(text: str):
    """-> (constants [(name, value)], structs [(name, [(ctype, field)])], funcs [(ret, name, [(ctype, pname)])])."""
    raw = text
    text = _strip_comments(text)
    consts = []
    for m in re.finditer(r"^#define\s+(CRDT_[A-Z_]+)\s+(-?0x[0-9a-fA-F]+u?|-?\d+)", raw, flags=re.M):
        name, val = m.group(1), m.group(2).rstrip("u")
        if name == "CRDT_GPU_H":
            continue
        consts.append((name, val))
    structs = []
    for m in re.finditer(r"typedef\s+struct\s+(\w+)\s*\{(.*?)\}\s*(\w+)\s*;", text, flags=re.S):
        sname, body = m.group(1), m.group(2)
        fields = []
        for stmt in body.split(";"):
            stmt = " ".join(stmt.split())
            if not stmt:
                continue
            fp = re.match(r"^(.*?)\(\s*\*\s*(\w+)\s*\)\s*\((.*)\)$", stmt)
            if fp:  # function pointer field: 'int (*allgather)(void *user, ...)'
                fields.append((f"{fp.group(1).strip()} (*)({fp.group(3).strip()})", fp.group(2)))
                continue
            # 'size_t G, R, M, A' and 'const uint64_t *def_clock'
            first, *rest = [x.strip() for x in stmt.split(",")]
            ctype, name = _split_decl(first)
            fields.append((ctype, name))
            base = ctype.replace("*", "").strip()
            for r in rest:
                stars = r.count("*")
                fields.append(((base + " " + "*" * stars).strip(), r.replace("*", "").strip()))
        structs.append((sname, fields))
    funcs = []
    for m in re.finditer(r"^([A-Za-z_][\w \t]*?\**)\s*\b(crdt_\w+)\s*\(([^;{]*?)\)\s*;", text, flags=re.M | re.S):
        ret, name, params = " ".join(m.group(1).split()), m.group(2), m.group(3)
        plist = []
        params = " ".join(params.split())
        if params and params != "void":
            for p in params.split(","):
                plist.append(_split_decl(p.strip()))
        funcs.append((ret, name, plist))
    return consts, structs, funcs


def parse_rust_ffi(text: str):
    """-> (structs {name: [(field, rust type)]}, funcs {name: ([rust param types], rust ret)})."""
    structs = {}
    for m in re.finditer(r"pub struct (\w+) \{(.*?)\n\}", text, flags=re.S):
        fields = []
        for line in m.group(2).splitlines():
            line = line.strip().rstrip(",")
            if line.startswith("pub "):
                f, t = line[4:].split(":", 1)
                fields.append((f.strip(), t.strip()))
        structs[m.group(1)] = fields
    funcs = {}
    for m in re.finditer(r"pub fn (\w+)\((.*?)\) -> ([^;]+);", text, flags=re.S):
        args = [a.split(":", 1)[1].strip() for a in m.group(2).split(", ") if a.strip()]
        funcs[m.group(1)] = (args, m.group(3).strip())
    return structs, funcs
