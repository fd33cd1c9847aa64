"""Static check of the Go shim (integration/go/render/gpu/renderer_gpu.go) against the C
headers, without a Go toolchain.

cgo resolves every `C.name` against the preamble's headers and requires EXACT types: a
C.int passed where the prototype says uint32_t, or a C.uint32_t stored into a double field,
does not compile. This module translates the shim's C-facing statements into C++ that
compiles only when the same holds:

* every `C.izpi_*` call becomes a call through `cgo_call(fn, args...)`, a template that
  static_asserts the arity and that each argument's type equals the parameter's type
  (pointee const-ness ignored, as cgo does; untyped constants and nil accepted where cgo
  accepts them);
* every assignment to a field of a C struct (`r.req.width = C.uint32_t(...)`) asserts the
  field's type equals the value's;
* every field read (`desc.camera.exposure`, `st[i].rays`) must exist;
* every `C.IZPI_*` constant, `C.izpi_*` type and `C.izpi_*` function must be declared.

The C++ is compiled with g++ -fsyntax-only against include/. The translator knows the Go
subset the shim uses; a statement outside it is an error, so a later edit of the shim
either stays checkable or fails the test loudly.
"""
import re
import subprocess
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
SHIM = ROOT / "integration" / "go" / "render" / "gpu" / "renderer_gpu.go"

SCALARS = {"uint32_t", "uint64_t", "int", "double", "size_t", "char", "uint8_t", "int32_t", "int64_t"}
GO_ELEM = {"float64": "double", "uint32": "uint32_t", "byte": "unsigned char", "int": "long long",
           "uint64": "uint64_t"}

PRELUDE = r"""
#include <cstdint>
#include <cstdlib>
#include <type_traits>
#include "izpi_gpu.h"
#include "izpi_host.h"
// untyped Go constants (numbers, enum / #define constants): cgo converts them to the target type
struct untyped_int { long long v; template <class T> constexpr operator T() const { return (T)v; } };
constexpr untyped_int operator|(untyped_int a, untyped_int b) { return {a.v | b.v}; }
constexpr untyped_int operator+(untyped_int a, untyped_int b) { return {a.v + b.v}; }
constexpr untyped_int operator*(untyped_int a, untyped_int b) { return {a.v * b.v}; }
struct untyped_nil { template <class T> constexpr operator T*() const { return nullptr; } };
// cgo drops C qualifiers at every level: const T** is **C.T on the Go side
template <class T> struct cgo_norm { typedef typename std::remove_cv<T>::type type; };
template <class T> struct cgo_norm<T*> { typedef typename cgo_norm<typename std::remove_cv<T>::type>::type* type; };
template <class T> struct cgo_norm<T* const> { typedef typename cgo_norm<T*>::type type; };
template <class P, class A> constexpr bool cgo_same() {
  typedef typename std::decay<A>::type D;
  if (std::is_same<D, untyped_int>::value) return std::is_arithmetic<P>::value || std::is_enum<P>::value;
  if (std::is_same<D, untyped_nil>::value) return std::is_pointer<P>::value;
  return std::is_same<typename cgo_norm<P>::type, typename cgo_norm<D>::type>::value;
}
template <class R, class... P, class... A> R cgo_call(R (*)(P...), A&&...) {
  static_assert(sizeof...(P) == sizeof...(A), "cgo: argument count differs from the prototype");
  static_assert((cgo_same<P, A>() && ...), "cgo: argument type differs from the prototype");
  return R();
}
template <class F, class V> void cgo_assign(F& field, V&&) {
  static_assert(cgo_same<F, V>(), "cgo: value type differs from the field type");
}
template <class T> T& deref(T* p) { return *p; }
template <class T> T& deref(T& v) { return v; }
inline int gostring(const char*) { return 0; }
"""


class Untranslatable(Exception):
    pass


def _split_top(s, sep=","):
    out, depth, cur, quote = [], 0, "", False
    for ch in s:
        if ch == '"':
            quote = not quote
        if not quote:
            if ch in "([{":
                depth += 1
            elif ch in ")]}":
                depth -= 1
        if ch == sep and depth == 0 and not quote:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def _match_paren(s, i):
    """index of the ')' matching the '(' at s[i]"""
    depth = 0
    for j in range(i, len(s)):
        if s[j] == "(":
            depth += 1
        elif s[j] == ")":
            depth -= 1
            if depth == 0:
                return j
    raise Untranslatable("unbalanced parentheses: " + s)


class Translator:
    """Go expression (the shim's subset) -> (C++ text, touches C)."""

    def __init__(self, env):
        self.env = env  # local name -> C++ declaration kind ("var", "array", "field")

    def expr(self, s):
        s = s.strip()
        parts = _split_binop(s)
        if len(parts) > 1:
            outs = [self.expr(p) for p in parts[::2]]
            if not any(c for _, c in outs):
                return "untyped_int{0}", False
            return "(" + " ".join(t if i % 2 else outs[i // 2][0] for i, t in enumerate(parts)) + ")", True
        return self.unary(s)

    def unary(self, s):
        s = s.strip()
        if s.startswith("&"):
            t, c = self.unary(s[1:])
            return "&" + t, c
        if s == "nil":
            return "untyped_nil{}", False
        if re.fullmatch(r"-?\d+(\.\d+)?", s):
            return "untyped_int{%s}" % s.split(".")[0], False
        if s.startswith('"'):
            return "0", False
        m = re.match(r"\(\*C\.(\w+)\)\((.*)\)$", s)
        if m and _match_paren(s, s.index("(", 2)) == len(s) - 1:
            inner, c = self.expr(m.group(2))
            return "((%s*)(%s))" % (m.group(1), inner if c else "(void*)0"), True
        if s.startswith("(") and _match_paren(s, 0) == len(s) - 1:
            t, c = self.expr(s[1:-1])
            return "(" + t + ")", c
        # primary: a dotted name, then postfix calls / indexes / selectors
        m = re.match(r"[A-Za-z_]\w*(\.[A-Za-z_]\w*)*", s)
        if not m:
            raise Untranslatable(s)
        name, rest = m.group(0), s[m.end():]
        if rest.startswith("("):
            j = _match_paren(rest, 0)
            args, rest = rest[1:j], rest[j + 1:]
            t, c = self.call(name, args)
        else:
            t, c = self.name(name)
        while rest:
            if rest.startswith("["):
                j = rest.index("]")
                idx = rest[1:j]
                t = "%s[0]" % t if re.fullmatch(r"\w+", idx) else None
                if t is None:
                    raise Untranslatable(s)
                rest = rest[j + 1:]
            elif rest.startswith("."):
                m2 = re.match(r"\.(\w+)", rest)
                t = "deref(%s).%s" % (t, m2.group(1))
                rest = rest[m2.end():]
            elif rest.startswith("("):  # method call on a Go value (e.g. b.Dx())
                j = _match_paren(rest, 0)
                if c:
                    raise Untranslatable(s)
                rest = rest[j + 1:]
            else:
                raise Untranslatable(s)
        return t, c

    def name(self, name):
        if name.startswith("C."):
            n = name[2:]
            if n.startswith("IZPI_"):
                return "untyped_int{%s}" % n, True
            raise Untranslatable(name)
        head, *tail = name.split(".")
        if head == "r" and tail:
            t = "r->" + tail[0]
            for f in tail[1:]:
                t = "deref(%s).%s" % (t, f)
            return t, True
        if head in self.env:
            t = head
            for f in tail:
                t = "deref(%s).%s" % (t, f)
            return t, True
        return "untyped_int{0}", False  # a Go value (opt.SizeX, n, i, ...)

    def call(self, name, args):
        a = _split_top(args) if args.strip() else []
        if name.startswith("C."):
            f = name[2:]
            if f in SCALARS:
                inner = [self.expr(x) for x in a]
                pre = "".join("(void)(%s), " % t for t, c in inner if c)
                return "(%s(%s)0)" % (pre, f), True
            if f == "CString":
                return "((char*)0)", True
            if f == "GoString":
                t, _ = self.expr(a[0])
                return "gostring(%s)" % t, True
            if f in ("malloc", "free"):
                inner = [self.expr(x) for x in a]
                return "%s(%s)" % (f, ", ".join(t for t, _ in inner)), True
            if f.startswith("izpi_"):
                inner = [self.expr(x)[0] for x in a]
                return "cgo_call(&%s%s)" % (f, "".join(", " + t for t in inner)), True
            raise Untranslatable(name)
        if name == "unsafe.Pointer":
            t, c = self.expr(a[0])
            return "((void*)(%s))" % t, c
        if name == "unsafe.Add":
            p, _ = self.expr(a[0])
            return "((void*)((char*)(%s) + 1))" % p, True
        if name == "unsafe.Slice":
            return "untyped_int{0}", False
        inner = [self.expr(x) for x in a]
        if name in ("int", "int64", "uint64", "float64", "uint32") and inner and inner[0][1]:
            return "((long long)(%s))" % inner[0][0], True
        if any(c for _, c in inner):
            # a Go function of C values: keep the C expressions checked
            return "(%s, untyped_int{0})" % ", ".join("(void)(%s)" % t for t, c in inner if c), True
        return "untyped_int{0}", False


def _split_binop(s):
    """['a', '|', 'b', '+', 'c'] at depth 0 (binary | + * / only; no unary minus here)"""
    out, depth, cur = [], 0, ""
    i = 0
    while i < len(s):
        ch = s[i]
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if depth == 0 and ch in "|+*/" and cur.strip() and not (ch == "*" and cur.rstrip().endswith("(")):
            out += [cur.strip(), ch]
            cur = ""
        else:
            cur += ch
        i += 1
    out.append(cur.strip())
    return out if len(out) > 1 else [s]


def _go_type(t):
    """Go type -> (C++ declaration format with {} for the name, is_array)"""
    t = t.strip()
    if t.startswith("[]"):
        e = t[2:]
        e = e[2:] if e.startswith("C.") else GO_ELEM.get(e)
        if e is None:
            return None
        return e + " {}[1]", True
    if t.startswith("*C."):
        return t[3:] + "* {}", False
    if t.startswith("C."):
        return t[2:] + " {}", False
    return None


def _functions(src):
    """(name, body) of every top-level func"""
    out = []
    for m in re.finditer(r"^func (?:\([^)]*\) )?(\w+)\(", src, re.M):
        line = src[m.start():src.index("\n", m.start())]
        if line.rstrip().endswith("}"):  # one-line function
            out.append((m.group(1), line[line.index("{") + 1:line.rindex("}")]))
            continue
        start = src.index("{\n", m.end()) + 2
        end = src.index("\n}\n", start)
        out.append((m.group(1), src[start:end]))
    return out


def translate(src):
    """The C++ translation unit for the shim's source text."""
    lines = [PRELUDE]
    # the Renderer struct's fields
    sm = re.search(r"type Renderer struct \{(.*?)\n\}", src, re.S)
    fields = []
    for line in sm.group(1).splitlines():
        line = line.split("//")[0].strip()
        if not line:
            continue
        name, typ = line.split(None, 1)
        d = _go_type(typ)
        if d:
            fields.append(d[0].format(name) + ";")
    lines.append("struct R { %s };" % " ".join(fields))
    n = 0
    for fname, body in _functions(src):
        env, stmts = {}, []
        tr = Translator(env)
        joined, cur = [], ""
        for raw in body.splitlines():  # a statement continues while its parentheses are open
            cur += " " + raw.split("//")[0].strip()
            if cur.count("(") == cur.count(")"):
                joined.append(cur.strip())
                cur = ""
        for s in joined:
            if not s:
                continue
            if s.startswith("}"):  # Go blocks are C++ blocks: `:=` names keep their scope
                stmts.append("}")
                s = s[1:].strip()
                s = re.sub(r"^\(\)", "", s).strip()
            opens = s.endswith("{")
            if opens:
                s = s[:-1].strip()
            stmts += _statement(tr, env, s)
            if opens:
                stmts.append("{")
        n += 1
        lines.append("void f%d_%s() { R r_obj{}; R* r = &r_obj; (void)r;\n  %s\n}" % (n, fname, "\n  ".join(stmts)))
    return "\n".join(lines) + "\n"


def _statement(tr, env, s):
    """C++ statements checking one Go statement (a block opener without its brace)."""
    if not s:
        return []
    m = re.match(r"var (\w+(?:, \w+)*) (\S+)$", s)
    if m:
        d = _go_type(m.group(2))
        out = []
        for v in m.group(1).split(", ") if d else []:
            env[v] = "var"
            out.append(d[0].format(v) + "{};")
        return out
    m = re.match(r"(\w+) := make\((\[\][\w.]+),(.*)\)$", s)
    if m:
        d = _go_type(m.group(2))
        uses = _uses(tr, env, m.group(3))  # the length expression may call C
        if not d:
            return uses
        env[m.group(1)] = "array"
        return uses + [d[0].format(m.group(1)) + ";"]
    m = re.match(r"(\w+) := toFloat64NRGBA\(", s)
    if m:
        env[m.group(1)] = "array"
        return ["double %s[1];" % m.group(1)]
    m = re.match(r"(\w+), err := proto\.Marshal\(", s)
    if m:
        env[m.group(1)] = "array"
        return ["unsigned char %s[1];" % m.group(1)]
    m = re.match(r"(\w+) := (.*\bC\..*|r\.req)$", s)
    if m and not s.startswith("if "):
        t, _ = tr.expr(m.group(2))
        env[m.group(1)] = "var"
        return ["auto %s = %s;" % (m.group(1), t)]
    # assignments to C struct fields (r.req.x, req.x), single or multiple
    m = re.match(r"((?:r\.)?req\.[^=:!<>]*?)\s*=\s*([^=].*)$", s)
    if m and "C." not in m.group(1):
        lhs, rhs = _split_top(m.group(1)), _split_top(m.group(2))
        if len(lhs) != len(rhs):
            raise Untranslatable(s)
        out = []
        for lv, rv in zip(lhs, rhs):
            lt, _ = tr.expr(lv.replace("[i]", "[0]"))
            rt, _ = tr.expr(rv)
            out.append("cgo_assign(%s, %s);" % (lt, rt))
        return out
    return _uses(tr, env, s)


def _uses(tr, env, s):
    """Checks of the C calls, field reads, constants and types one Go statement names."""
    out = []
    # every C call, checked where it stands (a nested call is checked inside its caller)
    for cm in re.finditer(r"C\.(izpi_\w+)\(", s):
        if cm.start() > 0 and re.match(r"[\w.]", s[cm.start() - 1]):
            continue
        j = _match_paren(s, cm.end() - 1)
        call = s[cm.start():j + 1]
        if any(call in prev for prev in out):
            continue
        t, _ = tr.expr(call)
        out.append("(void)%s;" % t)
    # field reads of C structs through locals (desc.num_tris, st[i].rays)
    for fm in re.finditer(r"\b(\w+)(\[i\])?\.(\w+)", s):
        if env.get(fm.group(1)):
            b = fm.group(1) + ("[0]" if fm.group(2) else "")
            out.append("(void)deref(%s).%s;" % (b, fm.group(3)))
    # C constants and types named anywhere
    for cm in re.finditer(r"C\.(IZPI_\w+)", s):
        out.append("(void)(%s);" % cm.group(1))
    for cm in re.finditer(r"C\.(izpi_\w+)\b(?!\()", s):
        out.append("(void)sizeof(%s);" % cm.group(1))
    return out


def check(src, cxx="g++"):
    """(ok, compiler output, C++ text)"""
    code = translate(src)
    with tempfile.TemporaryDirectory() as d:
        f = Path(d) / "shim_check.cpp"
        f.write_text(code)
        r = subprocess.run([cxx, "-std=c++17", "-fsyntax-only", "-Wno-unused-value", "-I", str(ROOT / "include"), str(f)],
                           capture_output=True, text=True, timeout=120)
    return r.returncode == 0, r.stderr, code


if __name__ == "__main__":
    ok, err, code = check(SHIM.read_text())
    print(code)
    print("OK" if ok else err)
