"""A small C++-subset -> Python translator for straight-line and structured g2o control code,
used by gen_g2o_solver.py to evaluate the reference's own text (no reference source is
stored: the golden fixture is numbers only).

Object model: every member of the object whose method is translated lives in a dict `M`
(identifiers starting with `_` and the method's own calls), every other object is a dict of
callables (`a->b(x)` and `a.b(x)` become a['b'](x)).  Pointers to members are cells
(`&_x` -> _ref(M, '_x'), `*(p)` -> _deref(p), `*(p) = v` -> _deref_set(p, v)).  Members
declared `float` in the class are rounded to float32 on every assignment, as C++ does.

Supported statements: declarations (`T x = e;`, `T& x = e;`, `T* x = e;`), assignments
(= += -= *= /=), ++/--, calls, `if / else if / else` (with or without braces),
`for (init; cond; step)`, `do { } while (cond);`, `return [e];`.  Skipped: assert, cerr/cout
streams, preprocessor lines, G2O batch-statistics blocks.  Anything else raises.
The produced source is run through safe_exec (AST whitelist, no builtins).
"""
import re


class Unsupported(ValueError):
    pass


def function_body(src, signature):
    i = src.index(signature)
    j = src.index("{", i)
    depth, k = 0, j
    while True:
        if src[k] == "{":
            depth += 1
        elif src[k] == "}":
            depth -= 1
            if depth == 0:
                body = src[j + 1:k]
                break
        k += 1
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    body = re.sub(r"//[^\n]*", "", body)
    body = "\n".join(l for l in body.split("\n") if not l.strip().startswith("#"))
    return body


def member_types(header_src, class_name):
    """{member: c_type} of `class class_name { ... }` (simple `T name;` declarations)."""
    i = header_src.index("class " + class_name) if ("class " + class_name) in header_src else \
        header_src.index("class  " + class_name)
    j = header_src.index("{", i)
    depth, k = 0, j
    while True:
        if header_src[k] == "{":
            depth += 1
        elif header_src[k] == "}":
            depth -= 1
            if depth == 0:
                break
        k += 1
    out = {}
    for m in re.finditer(r"\b(float|double|int|bool)\s+(_?\w+)\s*;", header_src[j:k]):
        out[m.group(2)] = m.group(1)
    return out


# ------------------------------------------------------------------------------ tokenizer
def _split_statements(body):
    """Yield top-level statements / compound statements as (kind, text) with nested bodies."""
    s = body
    i, n = 0, len(s)
    out = []
    while i < n:
        while i < n and s[i] in " \t\r\n;":
            i += 1
        if i >= n:
            break
        start = i
        m = re.match(r"(if|for|while|do|else)\b", s[i:])
        if m:
            kw = m.group(1)
            i += len(kw)
            if kw in ("if", "for", "while"):
                while s[i] in " \t\r\n":
                    i += 1
                assert s[i] == "(", s[start:start + 40]
                i = _match(s, i, "(", ")")
            # statement body: block or single statement
            while i < n and s[i] in " \t\r\n":
                i += 1
            if kw == "else" and re.match(r"if\b", s[i:]):
                # else if: the whole following if statement (with its own else chain)
                L = _stmt_len(s[i:])
                out.append(("else", "else", _split_statements(s[i:i + L])))
                i += L
                continue
            j = i
            if s[j] == "{":
                j = _match(s, j, "{", "}")
                blk = s[i + 1:j - 1]
            else:
                j = _stmt_end(s, j) + 1
                blk = s[i:j]
            if kw == "do":
                # do { } while (cond);
                k = j
                while s[k] in " \t\r\n":
                    k += 1
                mm = re.match(r"while\s*", s[k:])
                assert mm, "do without while"
                k += mm.end()
                e = _match(s, k, "(", ")")
                cond = s[k + 1:e - 1]
                k = e
                while s[k] in " \t\r\n":
                    k += 1
                assert s[k] == ";"
                out.append(("do", cond, _split_statements(blk)))
                i = k + 1
                continue
            header = s[start:i].strip()
            out.append((kw, header, _split_statements(blk)))
            i = j
            continue
        j = _stmt_end(s, i)
        out.append(("stmt", " ".join(s[start:j].split()), None))
        i = j + 1
    return out


def _stmt_len(s):
    """Length of one statement (if / compound / simple) at the start of s."""
    i = 0
    while s[i] in " \t\r\n":
        i += 1
    m = re.match(r"(if|for|while)\b", s[i:])
    if m:
        i += len(m.group(1))
        while s[i] in " \t\r\n":
            i += 1
        i = _match(s, i, "(", ")")
        while s[i] in " \t\r\n":
            i += 1
        if s[i] == "{":
            i = _match(s, i, "{", "}")
        else:
            i = _stmt_end(s, i) + 1
        k = i
        while k < len(s) and s[k] in " \t\r\n":
            k += 1
        if re.match(r"else\b", s[k:]):
            k += 4
            return k + _stmt_len(s[k:])
        return i
    if s[i] == "{":
        return _match(s, i, "{", "}")
    return _stmt_end(s, i) + 1


def _match(s, i, o, c):
    assert s[i] == o
    depth = 0
    while True:
        if s[i] == o:
            depth += 1
        elif s[i] == c:
            depth -= 1
            if depth == 0:
                return i + 1
        i += 1


def _stmt_end(s, i):
    depth = 0
    while True:
        ch = s[i]
        if ch in "([":
            depth += 1
        elif ch in ")]":
            depth -= 1
        elif ch == ";" and depth == 0:
            return i
        i += 1


# ------------------------------------------------------------------------------ expressions
_TYPE = (r"(?:const\s+)?(?:unsigned\s+)?(?:typename\s+)?[A-Za-z_][\w:]*(?:<[^;=()]*?>)?"
         r"(?:\s*\*|\s*&)?")
_FUNCS = {"pow": "_pow", "fabs": "_fabs", "sqrt": "_sqrt", "g2o_isfinite": "_isfinite"}


class Translator:
    def __init__(self, members, float_members=(), int_members=(), locals_=()):
        self.members = set(members)
        self.float_members = set(float_members)
        self.int_members = set(int_members)
        self.locals = set(locals_)

    # -- expressions
    def expr(self, e):
        e = e.strip()
        e = re.sub(r"std::numeric_limits<double>::max\(\)", "_DBL_MAX", e)
        e = re.sub(r"std::numeric_limits<int>::max\(\)", "_INT_MAX", e)
        e = re.sub(r"OptimizationAlgorithm::(OK|Fail|Terminate)", r"'\1'", e)
        e = re.sub(r"(static|const|dynamic|reinterpret)_cast<[^>]*>", "", e)
        e = re.sub(r"\(std::(min|max)\)", r"_\1", e)
        e = re.sub(r"std::(min|max)\b", r"_\1", e)
        e = re.sub(r"G2OBatchStatistics::globalStats\(\)", "None", e)
        e = re.sub(r"\bget_monotonic_time\(\)", "_time()", e)
        for f, g in _FUNCS.items():
            e = re.sub(r"\b%s\s*\(" % f, g + "(", e)
        e = re.sub(r"\bmakeProperty<[^(]*>\s*\(", "makeProperty(", e)
        e = re.sub(r"\bG2OBatchStatistics::setGlobalStats\b", "_nop", e)
        e = re.sub(r"\b(OK|Fail|Terminate)\b(?!')", r"'\1'", e)
        e = e.replace("&&", " and ").replace("||", " or ")
        # &member (a pointer to a member: a cell), &local (the local itself)
        e = re.sub(r"(?<!&)&\s*(_\w+)", r"_ref(M, '\1')", e)
        e = re.sub(r"(?<!&)&\s*([A-Za-z]\w*)", r"\1", e)
        # member access a->b / a.b (not numbers)
        e = re.sub(r"->\s*(\w+)", r"['\1']", e)
        e = re.sub(r"(?<=[\w\)\]])\.(?=[A-Za-z_])(\w+)", r"['\1']", e)
        # numeric literals like 1. or 2.
        e = re.sub(r"(?<![\w.])(\d+)\.(?![\d\w])", r"\1.0", e)
        # identifiers: members -> M['x'], unknown bare calls -> M['f']
        out = []
        for tok in re.split(r"('[^']*'|\b[A-Za-z_]\w*\b)", e):
            if not tok:
                continue
            if tok.startswith("'"):
                out.append(tok)
            elif re.fullmatch(r"[A-Za-z_]\w*", tok):
                out.append(tok)
            else:
                out.append(tok)
        e = "".join(out)
        e = self._names(e)
        e = e.replace("&&", " and ").replace("||", " or ")
        e = re.sub(r"!(?!=)", " not ", e)
        e = re.sub(r"\btrue\b", "True", e)
        e = re.sub(r"\bfalse\b", "False", e)
        e = re.sub(r"\bthis\b", "None", e)
        return " ".join(e.split())

    _KEEP = {"_pow", "_fabs", "_sqrt", "_isfinite", "_min", "_max", "_time", "_ref", "_deref", "_nop",
             "cerr", "endl",
             "_DBL_MAX", "_INT_MAX", "_f32", "_deref_set", "None", "True", "False", "M", "and", "or", "not", "true", "false", "this"}

    def _names(self, e):
        def rep(m):
            name = m.group(0)
            start = m.start()
            prev = e[:start].rstrip()
            if prev.endswith("['") or prev.endswith("'"):
                return name
            if name in self._KEEP or name in self.locals:
                return name
            if name in self.members or name.startswith("_"):
                return "M['%s']" % name
            # a free function / method of the object -> M
            rest = e[m.end():].lstrip()
            if rest.startswith("("):
                return "M['%s']" % name
            return name
        return re.sub(r"(?<!['\w])[A-Za-z_]\w*(?![\w'])", rep, e)

    # -- statements
    def stmts(self, items, ind):
        lines = []
        i = 0
        while i < len(items):
            kind, head, sub = items[i]
            pad = "    " * ind
            if kind == "stmt":
                lines += [pad + x for x in self.simple(head)]
            elif kind == "if":
                cond = head[head.index("(") + 1:head.rindex(")")]
                lines.append(pad + "if %s:" % self.expr(cond))
                lines += self.block(sub, ind + 1)
                # else chain
                while i + 1 < len(items) and items[i + 1][0] == "else":
                    i += 1
                    lines.append(pad + "else:")
                    lines += self.block(items[i][2], ind + 1)
            elif kind == "for":
                inner = head[head.index("(") + 1:head.rindex(")")]
                init, cond, step = [x.strip() for x in _split_top(inner, ";")]
                lines += [pad + x for x in self.simple(init)]
                lines.append(pad + "while %s:" % self.expr(cond))
                lines += self.block(sub, ind + 1, tail=self.simple(step))
            elif kind == "do":
                lines.append(pad + "while True:")
                lines += self.block(sub, ind + 1)
                lines.append(pad + "    if not (%s):" % self.expr(head))
                lines.append(pad + "        break")
            elif kind == "else":
                raise Unsupported("dangling else")
            else:
                raise Unsupported(kind)
            i += 1
        return lines

    def block(self, sub, ind, tail=()):
        body = self.stmts(sub, ind)
        body += ["    " * ind + x for x in tail]
        if not body:
            body = ["    " * ind + "pass"]
        return body

    def simple(self, s):
        s = s.strip().rstrip(";").strip()
        s = re.sub(r"(static|const|dynamic|reinterpret)_cast<[^>]*>", "", s)
        if not s:
            return []
        if re.match(r"(assert|cerr|cout)\b", s) or s.startswith("std::cerr"):
            return []
        if "<<" in s and ("cerr" in s or "endl" in s):
            return []
        m = re.fullmatch(r"return\s*(.*)", s)
        if m:
            return ["return %s" % (self.expr(m.group(1)) if m.group(1) else "None")]
        m = re.fullmatch(r"(\+\+|--)\s*([\w>.-]+)", s) or re.fullmatch(r"([\w>.-]+)\s*(\+\+|--)", s)
        if m:
            g = m.groups()
            var, op = (g[1], g[0]) if g[0] in ("++", "--") else (g[0], g[1])
            return ["%s %s= 1" % (self.lhs(var), "+" if op == "++" else "-")]
        m = re.fullmatch(r"(%s)\s+(\w+)\s*=\s*(.+)" % _TYPE, s)     # declaration with init
        if m and not re.fullmatch(r"[\w>.\-\[\]]+", m.group(1).strip()) or \
                (m and m.group(1).split()[0] in ("int", "double", "bool", "float", "size_t", "const",
                                                 "OptimizationAlgorithm::SolverResult")) or \
                (m and ("*" in m.group(1) or "&" in m.group(1) or "::" in m.group(1))):
            name = m.group(2)
            self.locals.add(name)
            return ["%s = %s" % (name, self.cast(m.group(1), self.expr(m.group(3))))]
        m = re.fullmatch(r"(int|double|bool|float|size_t)\s+(\w+)", s)   # plain declaration
        if m:
            self.locals.add(m.group(2))
            return ["%s = 0" % m.group(2)]
        m = re.fullmatch(r"(\*\s*\(.+\))\s*=\s*(.+)", s)          # *(p) = v
        if m:
            inner = m.group(1).strip()[1:].strip()
            return ["_deref_set(%s, %s)" % (self.expr(inner[1:-1]), self.expr(m.group(2)))]
        m = re.fullmatch(r"([\w\[\]>.\-]+)\s*(=|\+=|-=|\*=|/=)\s*(.+)", s)
        if m:
            lhs = self.lhs(m.group(1))
            rhs = self.expr(m.group(3))
            name = m.group(1).strip()
            if m.group(2) == "=":
                return ["%s = %s" % (lhs, self.member_cast(name, rhs))]
            return ["%s = %s" % (lhs, self.member_cast(name, "(%s) %s (%s)" % (lhs, m.group(2)[0], rhs)))]
        if s.endswith(")") and not re.search(r"(?<![=!<>])=(?!=)", s):   # expression statement (call)
            return [self.expr(s)]
        raise Unsupported("statement: %s" % s)

    def lhs(self, v):
        return self.expr(v)

    def cast(self, ctype, rhs):
        t = ctype.replace("const", "").strip()
        if t == "float":
            return "_f32(%s)" % rhs
        return rhs

    def member_cast(self, name, rhs):
        if name in self.float_members:
            return "_f32(%s)" % rhs
        return rhs


def _split_top(s, sep):
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "([":
            depth += 1
        elif ch in ")]":
            depth -= 1
        if ch == sep and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    out.append(cur)
    return out


def translate(body, pyname, params, members=(), float_members=(), int_members=()):
    """-> Python source of `def pyname(M, *params)` for the C++ body."""
    tr = Translator(members, float_members, int_members, locals_=params)
    items = _split_statements(body)
    lines = tr.stmts(items, 1)
    if not lines:
        lines = ["    pass"]
    return "def %s(%s):\n%s\n" % (pyname, ", ".join(["M"] + list(params)), "\n".join(lines))
