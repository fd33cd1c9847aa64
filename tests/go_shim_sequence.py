"""The Go shim's C call SEQUENCE against the C replay's, in every branch, without a Go
toolchain (verdict r4 item 5).

integration/c/go_shim_replay.c replays the C calls of integration/go/render/gpu/
renderer_gpu.go, and the GPU tests run the replay, so the drop-in's parity rests on the
replay issuing what the shim issues. This module reads both sources, parses the function
bodies that make a frame (Go: New, then Render or RenderTiles, then Close; C: main) into
statements, if-chains and loops, and walks them for each scenario

    multi   Options.Devices has several devices      (replay: --devices a,b)
    gpu_bvh Options.BVH == BVHGPU                    (replay: no --ref-bvh)
    tiles   the worker's RenderTiles, not Render     (replay: --tiles N)

collecting the library calls in evaluation order (a call's arguments before the call;
calls in an `if` condition before its body). A branch whose body returns at its top level
(a failed call, a bad argument) is the failure path and is not taken. Every other branch
whose body calls the library must be decided by the scenario through the condition tables
below: a condition missing from them is an error, so an edit of either source that adds
a branch fails the check until the table says what the branch means.

Calls left out of the comparison, with why:
  izpi_*last_error            failure paths' messages
  izpi_host_scene_desc        an accessor of the host scene (no effect)
  izpi_host_bvh_leaf_max      a pure function of the descriptor
  izpi_gpu_progress,
  izpi_gpu_multi_progress     the shim's progress goroutine (monitoring, concurrent)
  izpi_scene_info,
  izpi_scene_image_file,
  izpi_host_tiles             what the replay reads to stand in for what the shim's caller
                              hands it (the leader's texture map, the worker's tile list)
"""
import itertools
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
SHIM = ROOT / "integration" / "go" / "render" / "gpu" / "renderer_gpu.go"
REPLAY = ROOT / "integration" / "c" / "go_shim_replay.c"

EXCLUDED = {"izpi_host_last_error", "izpi_gpu_last_error", "izpi_gpu_multi_last_error", "izpi_host_scene_desc",
            "izpi_host_bvh_leaf_max", "izpi_gpu_progress", "izpi_gpu_multi_progress", "izpi_scene_info",
            "izpi_scene_image_file", "izpi_host_tiles"}

# condition (spaces removed) -> scenario predicate: a key of the scenario, "!key", or "true"
GO_CONDITIONS = {
    "len(opt.Devices)>1": "multi",          # New: one context per device through izpi_gpu_multi_*
    "opt.BVH==BVHGPU": "gpu_bvh",           # New: the GPU BVH4 build
    "n>0": "true",                          # New: the scene has primitives
    "r.m!=nil": "multi",                    # upload, Render, Close
    "r.ctx!=nil": "!multi",                 # Close: a multi renderer's r.ctx was cleared with r.m
    "r.host!=nil": "true",                  # Close
    "r.ps!=nil": "true",                    # Close
}
C_CONDITIONS = {
    "ndev>1": "multi",
    "!ref_bvh": "gpu_bvh",
    "np>0": "true",
    "m": "multi",
    "ntiles>0": "tiles",
}


def blank_strings_and_comments(src, lang):
    """The source with string/char literals' contents and comments replaced by spaces
    (same length, newlines kept), so that braces, parens and names inside them are ignored."""
    out, i, n = list(src), 0, len(src)
    while i < n:
        c = src[i]
        if src.startswith("//", i):
            j = src.find("\n", i)
            j = n if j < 0 else j
            for k in range(i, j):
                out[k] = " "
            i = j
        elif src.startswith("/*", i):
            j = src.index("*/", i) + 2
            for k in range(i, j):
                if out[k] != "\n":
                    out[k] = " "
            i = j
        elif c in "\"'" or (c == "`" and lang == "go"):
            j = i + 1
            while src[j] != c:
                j += 2 if (src[j] == "\\" and c != "`") else 1
            for k in range(i + 1, j):
                if out[k] != "\n":
                    out[k] = " "
            i = j + 1
        else:
            i += 1
    return "".join(out)


def match_close(s, i):
    """Index just past the bracket that closes the one at s[i]."""
    pairs = {"(": ")", "[": "]", "{": "}"}
    stack = []
    for j in range(i, len(s)):
        if s[j] in pairs:
            stack.append(pairs[s[j]])
        elif s[j] in ")]}":
            if not stack or stack.pop() != s[j]:
                raise ValueError("unbalanced at %d" % j)
            if not stack:
                return j + 1
    raise ValueError("unclosed bracket at %d" % i)


def function_body(src, header):
    """The text inside the braces of the function whose definition starts with `header`."""
    i = src.index(header) + len(header) - 1  # at the parameter list's "("
    i = match_close(src, i)
    while src[i] != "{":
        if src[i] == "(":
            i = match_close(src, i)
        else:
            i += 1
    return src[i + 1:match_close(src, i) - 1]


def parse(body, lang):
    """Statements of a block: ("stmt", text), ("if", [(cond, block)...], else_block|None),
    ("loop", header, block)."""
    nodes, i, n = [], 0, len(body)

    def skip_ws(k):
        while k < n and body[k] in " \t\r\n;":
            k += 1
        return k

    def simple_end(k):  # end of a simple statement starting at k
        depth = 0
        while k < n:
            ch = body[k]
            if ch in "([{":
                k = match_close(body, k)
                continue
            if lang == "c" and ch == ";" and depth == 0:
                return k + 1
            if lang == "go" and ch == "\n":
                prev = body[:k].rstrip()
                if not prev or prev[-1] not in ",(+-*/&|=.":
                    return k
            k += 1
        return n

    def block_at(k):  # a braced block, or (C) one statement
        k = skip_ws(k)
        if body[k] == "{":
            e = match_close(body, k)
            return parse(body[k + 1:e - 1], lang), e
        e = simple_end(k)
        return parse(body[k:e], lang), e

    def header_at(k):  # (header text, index of the body) after "if"/"for"
        if lang == "c":
            k = skip_ws(k)
            e = match_close(body, k)
            return body[k + 1:e - 1], e
        j = k
        while body[j] != "{":
            j = match_close(body, j) if body[j] in "([" else j + 1
        return body[k:j], j

    while True:
        i = skip_ws(i)
        if i >= n:
            return nodes
        word = re.match(r"[A-Za-z_]\w*", body[i:])
        word = word.group(0) if word else ""
        if word == "if":
            arms, els = [], None
            k = i + 2
            while True:
                cond, k = header_at(k)
                blk, k = block_at(k)
                arms.append((cond, blk))
                j = skip_ws(k)
                if not body.startswith("else", j):
                    break
                j = skip_ws(j + 4)
                if body.startswith("if", j) and not re.match(r"\w", body[j + 2]):
                    k = j + 2
                    continue
                els, k = block_at(j)
                break
            nodes.append(("if", arms, els))
            i = k
        elif word == "for":
            hdr, k = header_at(i + 3)
            blk, k = block_at(k)
            nodes.append(("loop", hdr, blk))
            i = k
        elif word in ("switch", "select"):
            raise ValueError("%s statements are outside the checked subset" % word)
        else:
            e = simple_end(i)
            nodes.append(("stmt", body[i:e].strip()))
            i = e


def calls(text, lang):
    """Library calls in `text` in evaluation order (a call completes after its arguments)."""
    pat = r"\bC\.(izpi_\w+)\s*\(" if lang == "go" else r"(?<![\w.])(izpi_\w+)\s*\("
    found = []
    for m in re.finditer(pat, text):
        found.append((match_close(text, m.end() - 1), m.group(1)))
    return [name for _, name in sorted(found) if name not in EXCLUDED]


def has_calls(nodes, lang):
    for nd in nodes:
        if nd[0] == "stmt" and calls(nd[1], lang):
            return True
        if nd[0] == "if" and (any(calls(c, lang) or has_calls(b, lang) for c, b in nd[1]) or
                              (nd[2] and has_calls(nd[2], lang))):
            return True
        if nd[0] == "loop" and has_calls(nd[2], lang):
            return True
    return False


def returns_at_top(nodes):
    return any(nd[0] == "stmt" and (nd[1].startswith("return") or nd[1].startswith("log.Fatal")) for nd in nodes)


def decide(cond, blk, lang, env):
    if returns_at_top(blk):
        return False  # the failure (or early-exit) path
    table = GO_CONDITIONS if lang == "go" else C_CONDITIONS
    key = re.sub(r"\s+", "", cond)
    if lang == "go" and ";" in key:
        key = key.split(";")[-1]
    if key not in table:
        if has_calls(blk, lang):
            raise KeyError("undecided %s condition %r guards library calls" % (lang, cond.strip()))
        return False
    p = table[key]
    return True if p == "true" else (not env[p[1:]] if p.startswith("!") else env[p])


def walk(nodes, lang, env, out):
    """Append the calls of `nodes` under scenario `env` to out; True if a return ended it."""
    for nd in nodes:
        if nd[0] == "stmt":
            out.extend(calls(nd[1], lang))
            if nd[1].startswith("return"):
                return True
        elif nd[0] == "if":
            taken = False
            for cond, blk in nd[1]:
                out.extend(calls(cond, lang))
                if decide(cond, blk, lang, env):
                    taken = True
                    if walk(blk, lang, env, out):
                        return True
                    break
            if not taken and nd[2] is not None and walk(nd[2], lang, env, out):
                return True
        elif nd[0] == "loop":
            sub = []
            walk(nd[2], lang, env, sub)
            if sub:
                out.append(("per item",) + tuple(sub))
    return False


SCENARIOS = [dict(zip(("multi", "gpu_bvh", "tiles"), v)) for v in itertools.product((False, True), repeat=3)]


def go_sequence(src, env):
    s = blank_strings_and_comments(src, "go")
    out = []
    walk(parse(function_body(s, "func New("), "go"), "go", env, out)
    frame = "func (r *Renderer) RenderTiles(" if env["tiles"] else "func (r *Renderer) Render("
    walk(parse(function_body(s, frame), "go"), "go", env, out)
    walk(parse(function_body(s, "func (r *Renderer) Close("), "go"), "go", env, out)
    return out


def c_sequence(src, env):
    s = blank_strings_and_comments(src, "c")
    out = []
    walk(parse(function_body(s, "int main("), "c"), "c", env, out)
    return out


def check(go_src=None, c_src=None):
    """[(scenario, go calls, c calls)] for the scenarios where the two differ."""
    go_src = SHIM.read_text() if go_src is None else go_src
    c_src = REPLAY.read_text() if c_src is None else c_src
    bad = []
    for env in SCENARIOS:
        g, c = go_sequence(go_src, env), c_sequence(c_src, env)
        if g != c:
            bad.append((env, g, c))
    return bad
