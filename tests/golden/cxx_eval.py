"""A typed C++-subset -> Python translator for evaluating the reference's own C++ text.

tests/golden/cxx_subset.py (round 4) handles g2o's straight-line control code with regular
expressions.  The extractor, matcher and LocalBA bodies need more of C++: typed arithmetic
(int division, float rounding, implicit conversions), std::vector / std::list / std::pair with
iterators, pointers and pointer arithmetic, references, value-semantics class objects, function-
like macros, the comma operator and conditional compilation.  This module tokenises, runs a
small preprocessor, parses statements and expressions, types every expression, and emits Python
that reproduces the C++ semantics for the subset it accepts; anything outside the subset
raises Unsupported (it never guesses).  The emitted source is then run by safe_exec (AST
whitelist, no builtins) against the runtime in cxx_rt.py.

Typing rules emitted (C++ usual arithmetic conversions):
  * int op int stays integral (`/` truncates, `%` takes the dividend's sign);
  * if either operand is double the operation is a double one; else if either is float the
    result is rounded to float after every operation (_f32), as the reference's float code;
  * every store to a typed lvalue converts: to int truncates toward zero, to float rounds to
    nearest, to double widens; conversions at calls follow the callee's parameter types;
  * class objects are copied on declaration / by-value passing / container insertion and
    assigned in place (C++ copy assignment), pointers and iterators are values.
Names: locals and parameters become `v_<name>`, members of the object `M['<name>']`, free
functions and translated methods `f_<name>`, file-level constants `c_<name>`.

Test infrastructure only (the golden generators).
"""
import re

from cxx_rt import env as rt_env  # noqa: F401  (the generators import both)


class Unsupported(ValueError):
    pass


# ==================================================================== types
class Ty:
    pass


class Prim(Ty):
    __slots__ = ("k",)

    def __init__(self, k):
        self.k = k

    def __eq__(self, o):
        return isinstance(o, Prim) and o.k == self.k

    def __hash__(self):
        return hash(("p", self.k))

    def __repr__(self):
        return self.k


class PtrT(Ty):
    __slots__ = ("to",)

    def __init__(self, to):
        self.to = to

    def __eq__(self, o):
        return isinstance(o, PtrT) and o.to == self.to

    def __hash__(self):
        return hash(("*", self.to))

    def __repr__(self):
        return "%r*" % (self.to,)


class Cls(Ty):
    __slots__ = ("name", "args")

    def __init__(self, name, args=()):
        self.name = name
        self.args = tuple(args)

    def __eq__(self, o):
        return isinstance(o, Cls) and o.name == self.name and o.args == self.args

    def __hash__(self):
        return hash(("c", self.name, self.args))

    def __repr__(self):
        return self.name + ("<%s>" % ",".join(map(repr, self.args)) if self.args else "")


INT, FLOAT, DOUBLE, BOOL, VOID, NULLT = (Prim("int"), Prim("float"), Prim("double"),
                                         Prim("bool"), Prim("void"), Prim("nullptr"))
ARITH = (INT, FLOAT, DOUBLE, BOOL)
_INT_NAMES = {"int", "unsigned", "signed", "long", "short", "char", "uchar", "size_t", "uint64_t",
              "int64_t", "uint32_t", "int32_t", "uint16_t", "int16_t", "uint8_t", "int8_t",
              "schar", "ushort", "uint", "ptrdiff_t"}
_QUALS = {"const", "static", "volatile", "typename", "struct", "inline", "register", "constexpr",
          "mutable", "extern"}
_KEYWORDS = {"if", "else", "for", "while", "do", "return", "break", "continue", "switch", "case",
             "default", "goto", "new", "delete", "sizeof", "true", "false", "this", "NULL",
             "nullptr", "operator", "using", "namespace", "template", "throw", "try", "catch"}
_STRIP_NS = ("cv::", "std::", "g2o::", "Eigen::")


def _strip(name):
    for p in _STRIP_NS:
        if name.startswith(p):
            name = name[len(p):]
    return name


def is_arith(t):
    return isinstance(t, Prim) and t.k in ("int", "float", "double", "bool")


def is_obj(t):
    """Mutable class objects (value semantics: copied on construction, assigned in place).
    VALUE_CLASSES (cv::Matx, time points) are immutable values in the runtime: rebinding them
    is their assignment."""
    return isinstance(t, Cls) and t.name not in ("iterator", "Ptr", "InputArray", "OutputArray",
                                                 "PointView", "Cell") and t.name not in VALUE_CLASSES


VALUE_CLASSES = {"Matx33d", "Matx44d", "Matx22d", "Matx", "HResClk::time_point"}


def elem_type(cont):
    """Element type of a container type (what an iterator dereferences to)."""
    if cont.name in ("map", "unordered_map"):
        return Cls("pair", (cont.args[0], cont.args[1]))
    return cont.args[0]


_VEC_NAMES = {"Vec2d": (2, DOUBLE), "Vec3d": (3, DOUBLE), "Vec4d": (4, DOUBLE), "Vec2f": (2, FLOAT),
              "Vec3f": (3, FLOAT), "Vector2d": (2, DOUBLE), "Vector3d": (3, DOUBLE)}


def arith_result(a, b):
    if a == DOUBLE or b == DOUBLE:
        return DOUBLE
    if a == FLOAT or b == FLOAT:
        return FLOAT
    return INT


# ==================================================================== tokens + preprocessor
_TOKRE = re.compile(r"""
 (?P<ws>\s+)
|(?P<num>0[xX][0-9a-fA-F]+[uUlL]*|(?:\d+\.\d*|\.\d+|\d+)(?:[eE][+-]?\d+)?[fFuUlL]*)
|(?P<id>[A-Za-z_]\w*)
|(?P<str>"(?:\\.|[^"\\])*")
|(?P<chr>'(?:\\.|[^'\\])')
|(?P<op><<=|>>=|->|\+\+|--|<<|>>|<=|>=|==|!=|&&|\|\||\+=|-=|\*=|/=|%=|&=|\|=|\^=|::|[-+*/%&|^~!<>=?:;,.(){}\[\]#])
""", re.X)


class Tok:
    __slots__ = ("kind", "text")

    def __init__(self, kind, text):
        self.kind, self.text = kind, text

    def __repr__(self):
        return self.text


def tokenize(text):
    out, i = [], 0
    while i < len(text):
        m = _TOKRE.match(text, i)
        if not m:
            raise Unsupported("cannot tokenize at %r" % text[i:i + 30])
        i = m.end()
        k = m.lastgroup
        if k != "ws":
            out.append(Tok(k, m.group(k)))
    return out


def strip_comments(src):
    out, i, n = [], 0, len(src)
    while i < n:
        c = src[i]
        if c == '"' or c == "'":
            j = i + 1
            while j < n and src[j] != c:
                j += 2 if src[j] == "\\" else 1
            out.append(src[i:j + 1])
            i = j + 1
        elif src.startswith("//", i):
            j = src.find("\n", i)
            i = n if j < 0 else j
        elif src.startswith("/*", i):
            j = src.find("*/", i + 2)
            out.append(" " if src.count("\n", i, j) == 0 else "\n" * src.count("\n", i, j))
            i = n if j < 0 else j + 2
        else:
            out.append(c)
            i += 1
    return "".join(out)


def _pp_eval(toks, defined):
    """#if expression: defined(X) -> 0/1, other identifiers 0; || && ! ( ) and integers."""
    xs, i = [], 0
    while i < len(toks):
        t = toks[i]
        if t.text == "defined":
            if toks[i + 1].text == "(":
                xs.append("1" if toks[i + 2].text in defined else "0")
                i += 4
            else:
                xs.append("1" if toks[i + 1].text in defined else "0")
                i += 2
            continue
        if t.kind == "id":
            xs.append("0")
        elif t.kind == "num":
            xs.append(str(int(t.text.rstrip("uUlL"), 0)))
        elif t.text in ("&&", "||", "!", "(", ")"):
            xs.append({"&&": " and ", "||": " or ", "!": " not "}.get(t.text, t.text))
        else:
            raise Unsupported("#if operator %r" % t.text)
        i += 1
    expr = "".join(xs)
    if not re.fullmatch(r"[01()\s]*(?:(?:and|or|not)[01()\s]*)*", expr):
        raise Unsupported("#if expression %r" % expr)
    from safe_exec import safe_compile_eval, safe_eval
    return bool(safe_eval(safe_compile_eval(expr, "<pp>"), {}))


def preprocess(src, defined=(), macros=None):
    """Comments, line continuations, #define/#undef (object- and function-like), #if/#ifdef/
    #ifndef/#elif/#else/#endif; other directives are dropped.  -> token list."""
    macros = dict(macros or {})
    defined = set(defined)
    src = strip_comments(src).replace("\\\n", " ")
    out = []
    stack = []        # (active, taken)

    def active():
        return all(a for a, _ in stack)
    for line in src.split("\n"):
        s = line.strip()
        if s.startswith("#"):
            d = tokenize(s[1:])
            if not d:
                continue
            kw, rest = d[0].text, d[1:]
            if kw in ("if", "ifdef", "ifndef"):
                if not active():
                    stack.append((False, True))
                    continue
                if kw == "if":
                    v = _pp_eval(rest, defined | set(macros))
                elif kw == "ifdef":
                    v = rest[0].text in defined or rest[0].text in macros
                else:
                    v = not (rest[0].text in defined or rest[0].text in macros)
                stack.append((v, v))
            elif kw == "elif":
                a, taken = stack.pop()
                outer = all(x for x, _ in stack)
                v = outer and not taken and _pp_eval(rest, defined | set(macros))
                stack.append((v, taken or v))
            elif kw == "else":
                a, taken = stack.pop()
                stack.append((not taken, True))
            elif kw == "endif":
                stack.pop()
            elif kw == "define" and active():
                m = re.match(r"\s*#\s*define\s+(\w+)(\(([^)]*)\))?(.*)$", s)
                name, params, body = m.group(1), m.group(3), m.group(4)
                ps = None if m.group(2) is None else [p.strip() for p in params.split(",") if p.strip()]
                macros[name] = (ps, tokenize(body))
            elif kw == "undef" and active():
                macros.pop(rest[0].text, None)
            continue
        if active():
            out += expand(tokenize(line), macros)
    return out


def expand(toks, macros, hide=frozenset()):
    out, i = [], 0
    while i < len(toks):
        t = toks[i]
        if t.kind == "id" and t.text in macros and t.text not in hide:
            ps, body = macros[t.text]
            if ps is None:
                out += expand(body, macros, hide | {t.text})
                i += 1
                continue
            if i + 1 < len(toks) and toks[i + 1].text == "(":
                j, depth, args, cur = i + 2, 1, [], []
                while True:
                    x = toks[j]
                    if x.text in "([{" and x.kind == "op":
                        depth += 1
                    elif x.text in ")]}" and x.kind == "op":
                        depth -= 1
                        if depth == 0:
                            break
                    if x.text == "," and depth == 1:
                        args.append(cur)
                        cur = []
                    else:
                        cur.append(x)
                    j += 1
                args.append(cur)
                if ps == [] and args == [[]]:
                    args = []
                if len(args) != len(ps):
                    raise Unsupported("macro %s arity" % t.text)
                sub = []
                for b in body:
                    if b.kind == "id" and b.text in ps:
                        sub += args[ps.index(b.text)]
                    else:
                        sub.append(b)
                out += expand(sub, macros, hide | {t.text})
                i = j + 1
                continue
        out.append(t)
        i += 1
    return out


# ==================================================================== source helpers
def find_function(src, signature):
    """(params text, body text) of the definition starting with `signature` (a prefix up to and
    including the function name)."""
    i = src.index(signature)
    # a signature ending in "(" names the parameter list's own parenthesis (operator()( ...);
    # otherwise the first "(" of the matched header opens it
    j = i + len(signature) - 1 if signature.endswith("(") else src.index("(", i)
    depth, k = 0, j
    while True:
        if src[k] == "(":
            depth += 1
        elif src[k] == ")":
            depth -= 1
            if depth == 0:
                break
        k += 1
    params = src[j + 1:k]
    b = src.index("{", k)
    init = src[k + 1:b]
    depth, e = 0, b
    while True:
        if src[e] == "{":
            depth += 1
        elif src[e] == "}":
            depth -= 1
            if depth == 0:
                break
        e += 1
    return params, init, src[b + 1:e]


def class_body(src, name):
    m = re.search(r"\b(class|struct)\s+%s\b[^;{]*\{" % re.escape(name), src)
    if not m:
        raise Unsupported("class %s not found" % name)
    b = m.end() - 1
    depth, e = 0, b
    while True:
        if src[e] == "{":
            depth += 1
        elif src[e] == "}":
            depth -= 1
            if depth == 0:
                break
        e += 1
    return src[b + 1:e]


def int_array(src, name):
    """Numbers of `... name[...] = { ... };` (an initialised integer table)."""
    m = re.search(r"\b%s\s*\[[^\]]*\]\s*=\s*\{" % re.escape(name), src)
    if not m:
        raise Unsupported("array %s not found" % name)
    e = src.index("}", m.end())
    body = strip_comments(src[m.end():e])
    return [int(x) for x in re.findall(r"-?\d+", body)]


# ==================================================================== parser
class Parser:
    def __init__(self, toks, type_names=()):
        self.t = toks
        self.i = 0
        self.type_names = set(type_names)

    # -- token helpers
    def peek(self, k=0):
        j = self.i + k
        return self.t[j].text if j < len(self.t) else None

    def peekk(self, k=0):
        j = self.i + k
        return self.t[j].kind if j < len(self.t) else None

    def take(self, want=None):
        if self.i >= len(self.t):
            raise Unsupported("unexpected end (want %r)" % want)
        tok = self.t[self.i]
        if want is not None and tok.text != want:
            raise Unsupported("expected %r, got %r near %s" % (want, tok.text, self.ctx()))
        self.i += 1
        return tok

    def ctx(self):
        return " ".join(x.text for x in self.t[max(0, self.i - 6):self.i + 6])

    # -- types
    def try_type(self):
        """-> (Ty, is_ref) or None (position restored)."""
        save = self.i
        quals = []
        while self.peek() in _QUALS:
            quals.append(self.take().text)
        name = None
        ints = ("unsigned", "signed", "long", "short", "int", "char")
        if self.peek() in ints:                          # `long unsigned int`, `unsigned long`, ...
            while self.peek() in ints:
                self.take()
            name = "int"
            while self.peek() in _QUALS:
                self.take()
        elif self.peekk() == "id" and self.peek() not in _KEYWORDS:
            name = self.take().text
            while self.peek() == "::" and self.peekk(1) == "id":
                self.take()
                name += "::" + self.take().text
        if name is None:
            self.i = save
            return None
        base = _strip(name)
        self.last_base = base
        args = ()
        if self.peek() == "<" and self._templ_ok(base):
            args = self.template_args()
            while self.peek() == "::" and self.peekk(1) == "id":
                self.take()
                sub = self.take().text
                if sub in ("iterator", "const_iterator"):
                    base, args = "iterator", (Cls(base, args),)
                else:
                    raise Unsupported("nested type %s::%s" % (base, sub))
        ty = self.make_type(base, args)
        while self.peek() == "const":
            self.take()
        is_ref = False
        while self.peek() in ("*", "&", "const"):
            x = self.take().text
            if x == "*":
                ty = PtrT(ty)
            elif x == "&":
                is_ref = True
        return ty, is_ref

    def _templ_ok(self, base):
        return base in ("vector", "list", "pair", "Point_", "Ptr", "Matx", "Vec", "numeric_limits",
                        "set", "map", "unordered_map") or base in self.type_names

    def template_args(self):
        self.take("<")
        args = []
        while True:
            if self.peek() == ">":
                self.take()
                break
            if self.peek() == ">>":                      # C++11 `>>` closing two lists
                self.t[self.i:self.i + 1] = [Tok("op", ">"), Tok("op", ">")]
                continue
            if self.peekk() == "num":
                args.append(int(self.take().text.rstrip("uUlL")))
            else:
                r = self.try_type()
                if r is None:
                    raise Unsupported("template argument near %s" % self.ctx())
                args.append(PtrT(r[0]) if False else r[0])
            if self.peek() == ",":
                self.take()
        return tuple(args)

    @staticmethod
    def make_type(base, args=()):
        if base in _INT_NAMES:
            return INT
        if base == "float":
            return FLOAT
        if base == "double":
            return DOUBLE
        if base == "bool":
            return BOOL
        if base == "void":
            return VOID
        if base == "auto":
            return Cls("auto")
        if base == "Point":
            return Cls("Point2i")
        if base in ("Vec2d", "Vec3d", "Vec4d", "Vec2f", "Vec3f"):
            return Cls("Vec", (DOUBLE if base.endswith("d") else FLOAT, int(base[3])))
        return Cls(base, args)

    # -- statements
    def parse_body(self):
        out = []
        while self.i < len(self.t):
            out.append(self.statement())
        return out

    def statement(self):
        p = self.peek()
        if p == "{":
            self.take()
            body = []
            while self.peek() != "}":
                body.append(self.statement())
            self.take("}")
            return ("block", body)
        if p == ";":
            self.take()
            return ("block", [])
        if p == "if":
            self.take()
            self.take("(")
            c = self.expr()
            self.take(")")
            th = self.statement()
            el = None
            if self.peek() == "else":
                self.take()
                el = self.statement()
            return ("if", c, th, el)
        if p == "for":
            self.take()
            self.take("(")
            # range-for: for (T x : container)
            save = self.i
            r = self.try_type()
            if r is not None and self.peekk() == "id" and self.peek(1) == ":":
                name = self.take().text
                self.take(":")
                cont = self.expr()
                self.take(")")
                return ("rfor", r[0], r[1], name, cont, self.statement())
            self.i = save
            if self.peek() == ";":
                init = None
            else:
                init = self.decl_or_expr()
            self.take(";")
            cond = None if self.peek() == ";" else self.expr()
            self.take(";")
            step = None if self.peek() == ")" else self.expr()
            self.take(")")
            return ("for", init, cond, step, self.statement())
        if p == "while":
            self.take()
            self.take("(")
            c = self.expr()
            self.take(")")
            return ("while", c, self.statement())
        if p == "do":
            self.take()
            body = self.statement()
            self.take("while")
            self.take("(")
            c = self.expr()
            self.take(")")
            self.take(";")
            return ("do", body, c)
        if p in ("break", "continue"):
            self.take()
            self.take(";")
            return (p,)
        if p == "return":
            self.take()
            e = None if self.peek() == ";" else self.expr()
            self.take(";")
            return ("return", e)
        s = self.decl_or_expr()
        self.take(";")
        return s

    def decl_or_expr(self):
        save = self.i
        r = self.try_type()
        if r is not None and self.peekk() == "id" and self.peek() not in _KEYWORDS and \
                self.peek(1) in ("=", ";", ",", "(", "[", "{", ":"):
            return self.declarators(r)
        self.i = save
        return ("expr", self.expr())

    def declarators(self, r):
        base, is_ref = r
        decls = []
        while True:
            ty, ref = base, is_ref
            while self.peek() in ("*", "&"):     # `int a, *b` forms
                x = self.take().text
                if x == "*":
                    ty = PtrT(ty)
                else:
                    ref = True
            name = self.take().text
            dims = []
            while self.peek() == "[":
                self.take()
                dims.append(self.assign_expr())
                self.take("]")
            init = None
            if self.peek() == "=":
                self.take()
                init = ("=", self.assign_expr())
            elif self.peek() == "(":
                self.take()
                args = []
                while self.peek() != ")":
                    args.append(self.assign_expr())
                    if self.peek() == ",":
                        self.take()
                self.take(")")
                init = ("()", args)
            decls.append((ty, ref, name, dims, init))
            if self.peek() == ",":
                self.take()
                continue
            break
        return ("decl", decls)

    # -- expressions (precedence climbing)
    def expr(self):
        e = self.assign_expr()
        if self.peek() == ",":
            xs = [e]
            while self.peek() == ",":
                self.take()
                xs.append(self.assign_expr())
            return ("comma", xs)
        return e

    _ASSIGN = ("=", "+=", "-=", "*=", "/=", "%=", "&=", "|=", "^=", "<<=", ">>=")
    _BIN = [("||",), ("&&",), ("|",), ("^",), ("&",), ("==", "!="), ("<", ">", "<=", ">="),
            ("<<", ">>"), ("+", "-"), ("*", "/", "%")]

    def assign_expr(self):
        lhs = self.cond_expr()
        if self.peek() in self._ASSIGN:
            op = self.take().text
            rhs = self.assign_expr()
            return ("assign", op, lhs, rhs)
        return lhs

    def cond_expr(self):
        c = self.binary(0)
        if self.peek() == "?":
            self.take()
            a = self.assign_expr()
            self.take(":")
            b = self.assign_expr()
            return ("cond", c, a, b)
        return c

    def binary(self, lvl):
        if lvl == len(self._BIN):
            return self.unary()
        a = self.binary(lvl + 1)
        while self.peek() in self._BIN[lvl] and self.peekk() == "op":
            op = self.take().text
            b = self.binary(lvl + 1)
            a = ("bin", op, a, b)
        return a

    def unary(self):
        p = self.peek()
        if p in ("-", "+", "!", "~", "*", "&") and self.peekk() == "op":
            self.take()
            return ("un", p, self.unary())
        if p in ("++", "--"):
            self.take()
            return ("pre", p, self.unary())
        if p == "(":                                   # C cast?
            save = self.i
            self.take()
            r = self.try_type()
            if r is not None and self.peek() == ")" and self._is_cast_type(r[0]):
                self.take()
                if self.last_base in ("uchar", "uint8_t") and r[0] == INT:
                    return ("cast8", self.unary())
                return ("cast", r[0], self.unary())
            self.i = save
        return self.postfix()

    def _is_cast_type(self, ty):
        if isinstance(ty, PtrT):
            return True
        return isinstance(ty, Prim) or (isinstance(ty, Cls) and ty.name in self.type_names)

    def postfix(self):
        e = self.primary()
        while True:
            p = self.peek()
            if p == "(":
                self.take()
                args = []
                while self.peek() != ")":
                    args.append(self.assign_expr())
                    if self.peek() == ",":
                        self.take()
                self.take(")")
                e = ("call", e, args)
            elif p == "[":
                self.take()
                k = self.expr()
                self.take("]")
                e = ("index", e, k)
            elif p in (".", "->"):
                self.take()
                name = self.take().text
                targs = ()
                if self.peek() == "<" and name in ("at", "ptr"):
                    self.take("<")
                    raw = []
                    while self.peek() != ">":
                        raw.append(self.take().text)
                    self.take(">")
                    targs = (_strip("".join(raw)),)
                e = ("member", e, name, p == "->", targs)
            elif p in ("++", "--"):
                self.take()
                e = ("post", p, e)
            else:
                return e

    def primary(self):
        k, p = self.peekk(), self.peek()
        if k == "num":
            self.take()
            return ("num", p)
        if k == "chr":
            self.take()
            return ("num", str(ord(p[1:-1].encode().decode("unicode_escape"))))
        if k == "str":
            self.take()
            return ("str", p)
        if p == "(":
            self.take()
            e = self.expr()
            self.take(")")
            return ("paren", e)
        if k == "id" and p == "new":
            self.take()
            name = self.take().text
            while self.peek() == "::" and self.peekk(1) == "id":
                self.take()
                name += "::" + self.take().text
            if self.peek() == "<":                        # template arguments of the allocated type
                depth = 0
                while True:
                    t = self.take().text
                    depth += t.count("<") - t.count(">")
                    if depth <= 0:
                        break
            args = []
            if self.peek() == "(":
                self.take()
                while self.peek() != ")":
                    args.append(self.assign_expr())
                    if self.peek() == ",":
                        self.take()
                self.take(")")
            return ("new", _strip(name), args)
        if k == "id":
            name = self.take().text
            if name in ("static_cast", "const_cast", "reinterpret_cast", "dynamic_cast"):
                self.take("<")
                r = self.try_type()
                narrow = self.last_base in ("uchar", "uint8_t") and r[0] == INT
                self.take(">")
                self.take("(")
                e = self.expr()
                self.take(")")
                return ("cast8", e) if narrow else ("cast", r[0], e)
            while self.peek() == "::" and self.peekk(1) == "id":
                self.take()
                name += "::" + self.take().text
            base = _strip(name)
            if self.peek() == "<" and self._templ_ok(base) and base not in ("Ptr",):
                args = self.template_args()
                if self.peek() == "::":
                    self.take()
                    sub = self.take().text
                    return ("name", "%s<%s>::%s" % (base, ",".join(map(repr, args)), sub))
                return ("tname", base, args)
            return ("name", name)
        raise Unsupported("expression at %s" % self.ctx())


# ==================================================================== code generation
class Fn:
    """Signature of a callable the translated code may call."""

    def __init__(self, pyname, params, ret, method_of=None, defaults=()):
        self.pyname = pyname
        self.params = params          # [(Ty, is_ref, is_const)] or None (unchecked stand-in)
        self.ret = ret                # Ty, or a callable(arg types) -> Ty
        self.method_of = method_of
        self.defaults = list(defaults)   # Python code of the trailing default arguments


class ClassSpec:
    def __init__(self, name, fields=None, methods=None, ctor=None, smart=False, runtime_ctor=None):
        self.name = name
        self.fields = dict(fields or {})      # name -> Ty
        self.methods = dict(methods or {})    # name -> Fn (pyname None: a runtime method obj['m'])
        self.ctor = ctor                      # env name of the constructor callable
        self.smart = smart                    # `->` acts like `.` (cv::Ptr)
        self.runtime_ctor = runtime_ctor      # callable(*args) building the object (else a Struct)


class E:
    """A translated expression: code, type, lvalue store form (None | ('name', py) |
    ('sub', objcode, keycode) | ('cell', cellcode)), is a reference to an existing object."""
    __slots__ = ("code", "ty", "lv", "obj")

    def __init__(self, code, ty, lv=None, obj=False):
        self.code, self.ty, self.lv, self.obj = code, ty, lv, obj


class Ctx:
    """What the translator knows: classes, functions, constants."""

    def __init__(self):
        self.classes = {}      # name -> ClassSpec
        self.funcs = {}        # C++ name -> Fn
        self.consts = {}       # C++ name -> (pyname, Ty)
        self.type_names = set()
        self.factories = {}    # env name -> Ty of default elements the code constructs
        self.scalable = {}     # class name -> env helper for `object * scalar`

    def add_class(self, spec):
        self.classes[spec.name] = spec
        self.type_names.add(spec.name)


class FuncTranslator:
    def __init__(self, ctx, this_cls=None, ret=VOID):
        self.ctx = ctx
        self.this = this_cls           # ClassSpec of the object M, or None
        self.ret = ret
        self.scopes = [{}]             # C++ name -> (pyname, Ty, kind) kind: 'val' | 'ref' | 'cell'
        self.used = set()
        self.loops = []                # continue prefixes
        self.tmp = 0
        self.pre, self.post = [], []   # statements around the current one (out-parameters)

    # ---------------------------------------------------------------- scopes
    def declare(self, name, ty, kind="val"):
        py = "v_" + name
        k = 1
        while py in self.used and any(name in s for s in self.scopes):
            py = "v_%s_%d" % (name, k)
            k += 1
        self.used.add(py)
        self.scopes[-1][name] = (py, ty, kind)
        return py

    def lookup(self, name):
        for s in reversed(self.scopes):
            if name in s:
                return s[name]
        return None

    def newtmp(self):
        self.tmp += 1
        return "t_%d" % self.tmp

    # ---------------------------------------------------------------- conversions
    def conv(self, e, to):
        """Implicit / explicit conversion of E to type `to` -> code."""
        fr = e.ty
        if to == fr or to is None:
            return e.code
        if isinstance(to, Prim):
            if to == INT:
                if fr in (FLOAT, DOUBLE):
                    return "_trunc(%s)" % e.code
                if fr in (INT, BOOL):
                    return "(%s) + 0" % e.code if fr == BOOL else e.code
            if to == FLOAT:
                if fr in (INT, BOOL, DOUBLE):
                    return "_f32(%s)" % e.code
            if to == DOUBLE:
                if fr in (INT, BOOL):
                    return "_dbl(%s)" % e.code
                if fr == FLOAT:
                    return e.code
            if to == BOOL:
                if is_arith(fr):
                    return "((%s) != 0)" % e.code
                if isinstance(fr, PtrT) or fr == NULLT:
                    return "((%s) is not None)" % e.code
        if isinstance(to, PtrT):
            if fr == NULLT or (fr == INT and e.code in ("0",)):
                return "None"
            if isinstance(fr, PtrT):
                return e.code
        if isinstance(to, Cls) and isinstance(fr, Cls):
            if to.name == fr.name or to.name in ("InputArray", "OutputArray") or \
                    (to.name == "iterator" and fr.name == "iterator"):
                return e.code
        if isinstance(to, Cls) and to.name == "Mat" and fr == Cls("MatExpr"):
            return e.code
        if to == Cls("Point2d") and fr == Cls("Vec", (DOUBLE, 2)):
            # cv::Point_<double>(const Vec<double, 2>&): x = v[0], y = v[1] [ext, OpenCV types.hpp]
            return "_Point2d_vec(%s)" % e.code
        raise Unsupported("conversion %r -> %r of %s" % (fr, to, e.code))

    def store(self, lv, code):
        if lv is None:
            raise Unsupported("assignment to a non-lvalue")
        if lv[0] == "name":
            return "%s = %s" % (lv[1], code)
        if lv[0] == "sub":
            return "%s[%s] = %s" % (lv[1], lv[2], code)
        if lv[0] == "cell":
            return "%s[0] = %s" % (lv[1], code)
        raise Unsupported("store to %r" % (lv,))

    def default(self, ty, args_code=None):
        """Code constructing a default (or ctor-initialised) value of type ty."""
        if ty == INT or ty == BOOL:
            return "0" if ty == INT else "False"
        if ty in (FLOAT, DOUBLE):
            return "0.0"
        if isinstance(ty, PtrT):
            return "None"
        if isinstance(ty, Cls):
            if ty.name == "vector":
                return "_Vector(%s)" % self.factory(ty.args[0])
            if ty.name == "list":
                return "_List(%s)" % self.factory(ty.args[0])
            if ty.name in ("map", "unordered_map"):
                return "_Map(%s, %s)" % (self.factory(ty.args[1]), "True" if ty.name == "map" else "False")
            if ty.name == "pair":
                return "_Pair(%s, %s)" % (self.default(ty.args[0]), self.default(ty.args[1]))
            if ty.name == "iterator":
                return "None"
            if ty.name == "Vec":
                return "_VecN(%d)" % ty.args[1]
            spec = self.ctx.classes.get(ty.name)
            if spec is None or spec.ctor is None:
                raise Unsupported("no constructor for %r" % ty)
            return "%s()" % spec.ctor
        raise Unsupported("default of %r" % ty)

    def factory(self, ty):
        """Env name of a zero-argument callable making a default element."""
        key = "fac_" + re.sub(r"\W", "_", repr(ty))
        self.ctx.factories[key] = ty
        return key

    # ---------------------------------------------------------------- expressions
    def ex(self, n):
        k = n[0]
        m = getattr(self, "ex_" + k, None)
        if m is None:
            raise Unsupported("expression kind %s" % k)
        return m(n)

    def ex_paren(self, n):
        e = self.ex(n[1])
        return E("(%s)" % e.code, e.ty, e.lv, e.obj)

    def ex_num(self, n):
        t = n[1]
        if re.fullmatch(r"0[xX][0-9a-fA-F]+[uUlL]*", t):
            return E(str(int(t.rstrip("uUlL"), 16)), INT)
        if re.search(r"[.eE]", t) and not t.lower().startswith("0x"):
            if t[-1] in "fF":
                return E(repr(float(t[:-1])), FLOAT) if False else E("_f32(%r)" % float(t[:-1]), FLOAT)
            return E(repr(float(t.rstrip("lL"))), DOUBLE)
        return E(str(int(t.rstrip("uUlL"))), INT)

    def ex_str(self, n):
        return E(repr(n[1][1:-1]), Cls("str"))

    def ex_name(self, n):
        name = n[1]
        if name in ("true", "false"):
            return E("True" if name == "true" else "False", BOOL)
        if name in ("NULL", "nullptr"):
            return E("None", NULLT)
        if name == "this":
            return E("M", PtrT(Cls(self.this.name)))
        v = self.lookup(name)
        if v is not None:
            py, ty, kind = v
            if kind == "cell":
                return E("%s[0]" % py, ty, ("cell", py))
            return E(py, ty, ("name", py), obj=is_obj(ty))
        if self.this is not None:
            f = self.this.fields.get(name)
            if f is not None:
                return E("M[%r]" % name, f, ("sub", "M", repr(name)), obj=is_obj(f))
        s = _strip(name)
        if s in self.ctx.consts:
            py, ty = self.ctx.consts[s]
            return E(py, ty)
        raise Unsupported("unknown name %s" % name)

    def ex_un(self, n):
        op = n[1]
        if op == "&":
            return self.address_of(n[2])
        e = self.ex(n[2])
        if op == "*":
            if isinstance(e.ty, PtrT):
                to = e.ty.to
                if isinstance(to, Cls):
                    return E("_deref(%s)" % e.code, to, obj=is_obj(to))
                return E("%s[0]" % e.code, to, ("sub", e.code, "0"))
            if isinstance(e.ty, Cls) and e.ty.name == "iterator":
                to = elem_type(e.ty.args[0])
                if is_obj(to):
                    return E("_deref(%s)" % e.code, to, obj=True)
                return E("_deref(%s)" % e.code, to)
            raise Unsupported("dereference of %r" % e.ty)
        if op == "!":
            return E("(not %s)" % e.code, BOOL)
        if not is_arith(e.ty):
            raise Unsupported("unary %s on %r" % (op, e.ty))
        ty = INT if e.ty == BOOL else e.ty
        if op == "-":
            return E("(-%s)" % e.code, ty)
        if op == "+":
            return E(e.code, ty)
        if op == "~":
            if ty != INT:
                raise Unsupported("~ on %r" % ty)
            return E("(~%s)" % e.code, INT)
        raise Unsupported(op)

    def address_of(self, n):
        if n[0] == "paren":
            return self.address_of(n[1])
        if n[0] == "index":
            base = self.ex(n[1])
            k = self.ex(n[2])
            if isinstance(base.ty, Cls) and base.ty.name == "vector":
                return E("_addr_elem(%s, %s)" % (base.code, self.conv(k, INT)), PtrT(base.ty.args[0]))
            if isinstance(base.ty, PtrT):
                return E("(%s + %s)" % (base.code, self.conv(k, INT)), base.ty)
            raise Unsupported("address of element of %r" % base.ty)
        if n[0] == "call" and n[1][0] == "member" and n[1][2] == "at":
            obj = self.ex(n[1][1])
            args = [self.conv(self.ex(a), INT) for a in n[2]]
            return E("%s['addr_at'](%s)" % (obj.code, ", ".join(args)), PtrT(INT))
        e = self.ex(n)
        if is_obj(e.ty):
            return E("_addr(%s)" % e.code, PtrT(e.ty))
        if e.lv is not None and e.lv[0] == "name":
            raise Unsupported("address of a scalar local %s" % e.code)
        raise Unsupported("address of %r" % (n,))

    def ex_pre(self, n):
        raise Unsupported("++/-- inside an expression")

    def ex_post(self, n):
        raise Unsupported("++/-- inside an expression")

    def ex_cast(self, n):
        ty, e = n[1], self.ex(n[2])
        if isinstance(ty, PtrT) and e.ty == NULLT:
            return E("None", ty)
        if isinstance(ty, PtrT) and isinstance(e.ty, PtrT):
            if ty.to == Cls("Point2i") and e.ty.to == INT:
                return E("_PointView(%s)" % e.code, PtrT(Cls("Point2i")))
            if ty.to == e.ty.to or (ty.to == INT and e.ty.to == INT):
                return E(e.code, ty)
            if isinstance(ty.to, Cls) and isinstance(e.ty.to, Cls):
                return E(e.code, ty)              # static / dynamic cast between class pointers
            raise Unsupported("pointer cast %r -> %r" % (e.ty, ty))
        if isinstance(ty, Prim):
            if ty == INT and e.ty == INT:
                return E(e.code, INT)
            return E(self.conv(e, ty), ty)
        raise Unsupported("cast to %r" % ty)

    def ex_new(self, n):
        name, args = n[1], n[2]
        spec = self.ctx.classes.get(name)
        if spec is None or spec.ctor is None:
            raise Unsupported("new %s" % name)
        es = [self.ex(a) for a in args]
        return E("_addr(%s(%s))" % (spec.ctor, ", ".join(e.code for e in es)), PtrT(Cls(name)))

    def ex_cast8(self, n):
        e = self.ex(n[1])
        return E("((%s) & 255)" % self.conv(e, INT), INT)

    def ex_cond(self, n):
        c, a, b = self.ex(n[1]), self.ex(n[2]), self.ex(n[3])
        ty = a.ty
        if is_arith(a.ty) and is_arith(b.ty) and a.ty != b.ty:
            ty = arith_result(a.ty, b.ty)
        return E("(%s if %s else %s)" % (self.conv(a, ty), self.conv(c, BOOL), self.conv(b, ty)), ty)

    def ex_bin(self, n):
        op = n[1]
        a, b = self.ex(n[2]), self.ex(n[3])
        if op in ("&&", "||"):
            return E("(%s %s %s)" % (self.conv(a, BOOL), "and" if op == "&&" else "or", self.conv(b, BOOL)), BOOL)
        if op in ("==", "!=", "<", ">", "<=", ">="):
            if is_arith(a.ty) and is_arith(b.ty):
                return E("(%s %s %s)" % (a.code, op, b.code), BOOL)
            if op in ("==", "!="):
                if (isinstance(a.ty, PtrT) or a.ty == NULLT) and (isinstance(b.ty, PtrT) or b.ty == NULLT or b.code == "0"):
                    pb = "None" if b.ty != a.ty and (b.ty == NULLT or b.code == "0") else b.code
                    pa = a.code
                    if pb == "None":
                        return E("(%s %s None)" % (pa, "is" if op == "==" else "is not"), BOOL)
                    return E("(%s %s %s)" % (pa, op, pb), BOOL)
                if isinstance(a.ty, Cls) and a.ty.name == "iterator" and b.ty == a.ty:
                    return E("(%s %s %s)" % (a.code, op, b.code), BOOL)
            raise Unsupported("comparison %r %s %r" % (a.ty, op, b.ty))
        if isinstance(a.ty, Cls) and op == "*" and is_arith(b.ty) and a.ty.name in self.ctx.scalable:
            return E("%s(%s, %s)" % (self.ctx.scalable[a.ty.name], a.code, self.conv(b, DOUBLE)), a.ty)
        if isinstance(a.ty, PtrT) and op in ("+", "-") and is_arith(b.ty):
            return E("(%s %s %s)" % (a.code, op, self.conv(b, INT)), a.ty)
        if isinstance(a.ty, Cls) and a.ty.name == "iterator" and op in ("+", "-") and is_arith(b.ty):
            return E("(%s %s %s)" % (a.code, op, self.conv(b, INT)), a.ty)
        if not (is_arith(a.ty) and is_arith(b.ty)):
            raise Unsupported("operator %s on %r, %r" % (op, a.ty, b.ty))
        if op in ("&", "|", "^", "<<", ">>"):
            ta = INT if a.ty == BOOL else a.ty
            tb = INT if b.ty == BOOL else b.ty
            if ta != INT or tb != INT:
                raise Unsupported("bit operator on %r, %r" % (a.ty, b.ty))
            return E("(%s %s %s)" % (a.code, op, b.code), INT)
        r = arith_result(INT if a.ty == BOOL else a.ty, INT if b.ty == BOOL else b.ty)
        if r == INT:
            if op == "/":
                return E("_idiv(%s, %s)" % (a.code, b.code), INT)
            if op == "%":
                return E("_imod(%s, %s)" % (a.code, b.code), INT)
            return E("(%s %s %s)" % (a.code, op, b.code), INT)
        if op == "%":
            raise Unsupported("% on floating operands")
        ca, cb = self.conv(a, r) if a.ty != FLOAT else a.code, self.conv(b, r) if b.ty != FLOAT else b.code
        if r == DOUBLE:
            return E("(%s %s %s)" % (ca, op, cb), DOUBLE)
        # float: both operands are floats (ints converted exactly for |v| < 2^24), one rounding
        return E("_f32(%s %s %s)" % (ca, op, cb), FLOAT)

    def ex_index(self, n):
        base = self.ex(n[1])
        k = self.ex(n[2])
        ty = base.ty
        if isinstance(ty, Cls) and ty.name == "vector":
            el = ty.args[0]
            kc = self.conv(k, INT)
            return E("%s[%s]" % (base.code, kc), el, ("sub", base.code, kc), obj=is_obj(el))
        if isinstance(ty, Cls) and ty.name in ("map", "unordered_map"):
            el = ty.args[1]
            kc = self.conv(k, ty.args[0])
            return E("%s[%s]" % (base.code, kc), el, ("sub", base.code, kc), obj=is_obj(el))
        if isinstance(ty, Cls) and ty.name == "carray":
            el = ty.args[0]
            kc = self.conv(k, INT)
            return E("%s[%s]" % (base.code, kc), el, ("sub", base.code, kc), obj=is_obj(el))
        if isinstance(ty, PtrT):
            el = ty.to
            kc = self.conv(k, INT)
            return E("%s[%s]" % (base.code, kc), el, ("sub", base.code, kc), obj=is_obj(el))
        raise Unsupported("indexing %r" % ty)

    def member_type(self, ty, name):
        if isinstance(ty, Cls):
            if ty.name == "pair":
                return ty.args[0] if name == "first" else ty.args[1] if name == "second" else None
            spec = self.ctx.classes.get(ty.name)
            if spec is not None and name in spec.fields:
                return spec.fields[name]
        return None

    def ex_member(self, n):
        _, on, name, arrow, targs = n
        base = self.ex(on)
        ty = base.ty
        code = base.code
        if arrow:
            if isinstance(ty, PtrT):
                ty = ty.to
                code = "_deref(%s)" % code
            elif isinstance(ty, Cls) and ty.name == "iterator":
                ty = elem_type(ty.args[0])
                code = "_deref(%s)" % code
            elif isinstance(ty, Cls) and (ty.name == "Ptr" or self.ctx.classes.get(ty.name, ClassSpec("")).smart):
                ty = ty.args[0] if ty.name == "Ptr" else ty
            else:
                raise Unsupported("-> on %r" % ty)
        ft = self.member_type(ty, name)
        if ft is None:
            # a method: return a marker the call handles
            return E(code, ("method", ty, name, targs))
        return E("%s[%r]" % (code, name), ft, ("sub", code, repr(name)), obj=is_obj(ft))

    def ex_tname(self, n):
        return E(None, ("tname", n[1], n[2]))

    def ex_comma(self, n):
        raise Unsupported("comma operator inside an expression")

    def ex_assign(self, n):
        raise Unsupported("assignment inside an expression")

    # -- calls
    def take_prepost(self):
        p, q = self.pre, self.post
        self.pre, self.post = [], []
        return p, q

    def call_args(self, params, args):
        pre, post = self.pre, self.post
        out = []
        for i, a in enumerate(args):
            if params is None or i >= len(params):
                e = self.ex(a)
                out.append(e.code)
                continue
            pty, pref, pconst = params[i]
            e = self.ex(a)
            if pref and not pconst and isinstance(pty, Prim):
                # non-const scalar reference: pass a cell
                if e.lv is None:
                    raise Unsupported("scalar reference argument is not an lvalue")
                if e.lv[0] == "name":
                    t = self.newtmp()
                    pre.append("%s = [%s]" % (t, e.code))
                    post.append(self.store(e.lv, "%s[0]" % t))
                    out.append(t)
                elif e.lv[0] == "sub":
                    out.append("_Cell(%s, %s)" % (e.lv[1], e.lv[2]))
                elif e.lv[0] == "cell":
                    out.append(e.lv[1])
                else:
                    raise Unsupported("scalar reference argument %r" % (e.lv,))
                continue
            if is_obj(pty) and not pref:
                out.append("_cp(%s)" % self.conv(e, pty))
            elif isinstance(pty, Prim) or isinstance(pty, PtrT):
                out.append(self.conv(e, pty))
            else:
                out.append(self.conv(e, pty) if isinstance(e.ty, Ty) else e.code)
        return out

    def fill_defaults(self, fn, a):
        if fn.params is not None and len(a) < len(fn.params):
            need = len(fn.params) - len(a)
            if need > len(fn.defaults):
                raise Unsupported("too few arguments for %s" % fn.pyname)
            a = a + fn.defaults[len(fn.defaults) - need:]
        return a

    def ret_type(self, fn, argtys):
        return fn.ret(argtys) if callable(fn.ret) else fn.ret

    _MATH = {"sqrt": "_sqrt", "ceil": "_ceil", "floor": "_floor", "fabs": "_fabs", "abs": "_fabs",
             "pow": "_pow", "cos": "_cos", "sin": "_sin", "atan": "_atan", "atan2": "_atan2",
             "exp": "_exp", "log": "_log", "round": "_cround"}
    _EXACT_F = ("sqrt", "ceil", "floor", "fabs", "abs")   # float overloads equal to rounding the double result

    def ex_call(self, n):
        fnode, args = n[1], n[2]
        if fnode[0] == "member":
            base = self.ex(fnode)
            if not isinstance(base.ty, tuple):
                raise Unsupported("call of field %r" % (fnode,))
            _, oty, mname, targs = base.ty
            return self.method_call(base.code, oty, mname, targs, args)
        if fnode[0] == "tname":
            base, targs = fnode[1], fnode[2]
            if base in ("vector", "list", "map", "unordered_map") and len(args) == 0:
                ty = Cls(base, targs)
                return E(self.default(ty), ty, obj=True)
            if base == "vector" and len(args) in (1, 2):
                es = [self.ex(a) for a in args]
                if len(args) == 1:
                    return E("_vector_n(%s, %s)" % (self.factory(targs[0]), self.conv(es[0], INT)),
                             Cls("vector", targs), obj=True)
                return E("_vector_nv(%s, %s, %s)" % (self.factory(targs[0]), self.conv(es[0], INT),
                                                     self.conv(es[1], targs[0])), Cls("vector", targs), obj=True)
            raise Unsupported("call of template %s" % base)
        if fnode[0] != "name":
            e = self.ex(fnode)
            if isinstance(e.ty, Cls):                 # object call operator (Mat::operator())
                return self.method_call(e.code, e.ty, "()", (), args)
            raise Unsupported("call target %r" % (fnode,))
        name = fnode[1]
        s = _strip(name)
        # a method of the object being translated
        if self.this is not None and s in self.this.methods and self.lookup(s) is None:
            fn = self.this.methods[s]
            a = self.fill_defaults(fn, self.call_args(fn.params, args))
            return E("%s(%s)" % (fn.pyname, ", ".join(["M"] + a)), self.ret_type(fn, None))
        v = self.lookup(name)
        if v is not None and isinstance(v[1], Cls):
            return self.method_call(v[0], v[1], "()", (), args)
        if s in self._MATH and s not in self.ctx.funcs:
            es = [self.ex(a) for a in args]
            allf = all(e.ty == FLOAT for e in es)
            if allf and s not in self._EXACT_F:
                raise Unsupported("float overload of %s (libm float function)" % s)
            code = "%s(%s)" % (self._MATH[s], ", ".join(self.conv(e, DOUBLE) for e in es))
            if allf:
                return E("_f32(%s)" % code, FLOAT)
            if s in ("abs",) and all(e.ty == INT for e in es):
                raise Unsupported("integer abs")
            return E(code, DOUBLE)
        if s in self.ctx.funcs:
            fn = self.ctx.funcs[s]
            if fn.params is None:
                es = [self.ex(a) for a in args]
                return E("%s(%s)" % (fn.pyname, ", ".join(e.code for e in es)),
                         self.ret_type(fn, [e.ty for e in es]))
            argtys = None
            if callable(fn.ret):
                argtys = [self.ex(a).ty for a in args]
            a = self.fill_defaults(fn, self.call_args(fn.params, args))
            return E("%s(%s)" % (fn.pyname, ", ".join(a)), self.ret_type(fn, argtys))
        if s in _VEC_NAMES:
            n, et = _VEC_NAMES[s]
            es = [self.ex(a) for a in args]
            if len(es) != n:
                raise Unsupported("%s with %d values" % (s, len(es)))
            return E("_VecInit(%s)" % ", ".join(self.conv(e, et) for e in es), Cls("Vec", (et, n)), obj=True)
        if s in self.ctx.classes or s == "Point":
            cn = "Point2i" if s == "Point" else s
            spec = self.ctx.classes[cn]
            es = [self.ex(a) for a in args]
            return E("%s(%s)" % (spec.ctor, ", ".join(e.code for e in es)), Cls(cn), obj=True)
        raise Unsupported("unknown function %s" % name)

    def method_call(self, code, oty, mname, targs, args):
        if isinstance(oty, Cls) and oty.name in ("vector", "list"):
            el = oty.args[0]
            es = [self.ex(a) for a in args]
            if mname in ("size",):
                return E("%s['size']()" % code, INT)
            if mname == "empty":
                return E("%s['empty']()" % code, BOOL)
            if mname in ("push_back", "push_front"):
                return E("%s[%r](%s)" % (code, mname, self.conv(es[0], el)), VOID)
            if mname in ("front", "back"):
                return E("%s[%r]()" % (code, mname), el, None, obj=is_obj(el))
            if mname in ("begin", "end"):
                return E("%s[%r]()" % (code, mname), Cls("iterator", (oty,)))
            if mname in ("reserve", "clear", "pop_back"):
                return E("%s[%r](%s)" % (code, mname, ", ".join(self.conv(e, INT) for e in es)), VOID)
            if mname == "resize":
                a = [self.conv(es[0], INT)] + ([self.conv(es[1], el)] if len(es) > 1 else [])
                return E("%s['resize'](%s)" % (code, ", ".join(a)), VOID)
            if mname == "erase":
                return E("%s['erase'](%s)" % (code, ", ".join(e.code for e in es)), Cls("iterator", (oty,)))
            if mname == "insert":
                return E("%s['insert'](%s)" % (code, ", ".join(e.code for e in es)), VOID)
            raise Unsupported("%s::%s" % (oty.name, mname))
        if isinstance(oty, Cls) and oty.name in ("map", "unordered_map"):
            es = [self.ex(a) for a in args]
            if mname == "find":
                return E("%s['find'](%s)" % (code, self.conv(es[0], oty.args[0])), Cls("iterator", (oty,)))
            if mname == "count":
                return E("%s['count'](%s)" % (code, self.conv(es[0], oty.args[0])), INT)
            if mname in ("begin", "end"):
                return E("%s[%r]()" % (code, mname), Cls("iterator", (oty,)))
            if mname in ("size",):
                return E("%s['size']()" % code, INT)
            if mname == "empty":
                return E("%s['empty']()" % code, BOOL)
            if mname == "clear":
                return E("%s['clear']()" % code, VOID)
            raise Unsupported("map::%s" % mname)
        if isinstance(oty, Cls) and oty.name == "Vec" and mname == "()":
            es = [self.ex(a) for a in args]
            kc = self.conv(es[0], INT)
            return E("%s[%s]" % (code, kc), oty.args[0], ("sub", code, kc))
        cname = oty.name if isinstance(oty, Cls) else None
        spec = self.ctx.classes.get(cname)
        if spec is None or mname not in spec.methods:
            raise Unsupported("method %r::%s" % (oty, mname))
        fn = spec.methods[mname]
        a = self.fill_defaults(fn, self.call_args(fn.params, args))
        rt = self.ret_type(fn, None)
        if fn.pyname is None:            # runtime method: obj['name'](...)
            key = {"()": "call"}.get(mname, mname)
            if mname in ("at", "ptr") and targs:
                t = targs[0]             # the element type's name: ptr<uchar> / ptr<uint64_t> / at<double>
                et = {"uchar": INT, "uint8_t": INT, "uint64_t": INT, "int": INT, "double": DOUBLE,
                      "float": FLOAT}.get(t)
                if et is None:
                    raise Unsupported("Mat::%s<%s>" % (mname, t))
                rt = et if mname == "at" else PtrT(et)
                if t not in ("uchar", "uint8_t"):
                    key = "%s_%s" % (mname, t)
            return E("%s[%r](%s)" % (code, key, ", ".join(a)), rt, obj=is_obj(rt))
        return E("%s(%s)" % (fn.pyname, ", ".join([code] + a)), rt, obj=is_obj(rt))

    # ---------------------------------------------------------------- statements
    def st(self, n, ind):
        k = n[0]
        m = getattr(self, "st_" + k, None)
        if m is None:
            raise Unsupported("statement %s" % k)
        return m(n, ind)

    def block(self, stmts, ind, tail=()):
        self.scopes.append({})
        lines = []
        for s in stmts:
            lines += self.st(s, ind)
        self.scopes.pop()
        lines += ["    " * ind + x for x in tail]
        return lines or ["    " * ind + "pass"]

    def as_list(self, n):
        return n[1] if n[0] == "block" else [n]

    def st_block(self, n, ind):
        return self.block(n[1], ind)

    def st_if(self, n, ind):
        pad = "    " * ind
        e, pre, post = self.ex_full(n[1])
        c = self.conv(e, BOOL)
        if post:
            t = self.newtmp()
            pre = pre + ["%s = %s" % (t, c)] + post
            c = t
        lines = [pad + x for x in pre] + [pad + "if %s:" % c]
        lines += self.block(self.as_list(n[2]), ind + 1)
        if n[3] is not None:
            lines.append(pad + "else:")
            lines += self.block(self.as_list(n[3]), ind + 1)
        return lines

    def st_while(self, n, ind):
        pad = "    " * ind
        c, _ = self.cond(n[1], loop=True)
        self.loops.append([])
        lines = [pad + "while %s:" % c]
        lines += self.block(self.as_list(n[2]), ind + 1)
        self.loops.pop()
        return lines

    def st_do(self, n, ind):
        pad = "    " * ind
        self.scopes.append({})
        c, _ = self.cond(n[2], loop=True)
        check = ["if not %s:" % c, "    break"]
        self.scopes.pop()
        self.loops.append(check)
        lines = [pad + "while True:"]
        lines += self.block(self.as_list(n[1]), ind + 1, tail=check)
        self.loops.pop()
        return lines

    def st_for(self, n, ind):
        pad = "    " * ind
        _, init, cond, step, body = n
        self.scopes.append({})
        lines = []
        if init is not None:
            lines += self.st(init, ind)
        c = "True" if cond is None else self.cond(cond, loop=True)[0]
        steps = [] if step is None else self.expr_stmt(step, 0)
        self.loops.append(steps)
        lines.append(pad + "while %s:" % c)
        lines += self.block(self.as_list(body), ind + 1, tail=steps)
        self.loops.pop()
        self.scopes.pop()
        return lines

    def st_rfor(self, n, ind):
        """for (T x : c): x walks c's elements by iterator (vector, list, map)."""
        pad = "    " * ind
        _, ty, ref, name, cont_n, body = n
        c, pre, post = self.ex_full(cont_n)
        if post or not (isinstance(c.ty, Cls) and c.ty.name in ("vector", "list", "map", "unordered_map")):
            raise Unsupported("range-for over %r" % (c.ty,))
        el = elem_type(c.ty)
        self.scopes.append({})
        ct = self.newtmp()
        it = self.newtmp()
        lines = [pad + x for x in pre] + [pad + "%s = %s" % (ct, c.code), pad + "%s = %s['begin']()" % (it, ct)]
        lines.append(pad + "while %s != %s['end']():" % (it, ct))
        self.scopes.append({})
        if ty == Prim("auto") if False else False:
            pass
        vty = el if (isinstance(ty, Cls) and ty.name == "auto") else ty
        if ref:
            py = self.declare(name, vty, "ref" if is_obj(vty) else "val")
            head = ["%s = _deref(%s)" % (py, it)]
        else:
            py = self.declare(name, vty)
            head = ["%s = %s" % (py, ("_cp(_deref(%s))" if is_obj(vty) else "_deref(%s)") % it)]
        step = ["%s = _inc(%s)" % (it, it)]
        self.loops.append(step)
        inner = [pad + "    " + x for x in head]
        for st in self.as_list(body):
            inner += self.st(st, ind + 1)
        inner += [pad + "    " + x for x in step]
        self.loops.pop()
        self.scopes.pop()
        self.scopes.pop()
        return lines + inner

    def st_break(self, n, ind):
        return ["    " * ind + "break"]

    def st_continue(self, n, ind):
        pad = "    " * ind
        if not self.loops:
            raise Unsupported("continue outside a loop")
        return [pad + x for x in self.loops[-1]] + [pad + "continue"]

    def st_return(self, n, ind):
        pad = "    " * ind
        if n[1] is None:
            return [pad + "return None"]
        e, pre, post = self.ex_full(n[1])
        if post:
            raise Unsupported("out-parameters in a return expression")
        code = self.conv(e, self.ret) if isinstance(self.ret, Prim) else e.code
        return [pad + x for x in pre] + [pad + "return %s" % code]

    def ex_full(self, node):
        """Translate an expression with the statements its out-parameter calls need."""
        saved = self.take_prepost()
        e = self.ex(node)
        pre, post = self.take_prepost()
        self.pre, self.post = saved
        return e, pre, post

    def cond(self, node, loop=False):
        e, pre, post = self.ex_full(node)
        if post or (loop and pre):
            raise Unsupported("out-parameters in a condition")
        return self.conv(e, BOOL), pre

    def st_expr(self, n, ind):
        return ["    " * ind + x for x in self.expr_stmt(n[1], ind)]

    def expr_stmt(self, e, ind):
        """Statement-level expression -> lines (no indentation)."""
        k = e[0]
        if k == "paren":
            return self.expr_stmt(e[1], ind)
        if k == "comma":
            out = []
            for x in e[1]:
                out += self.expr_stmt(x, ind)
            return out
        if k in ("pre", "post"):
            t = self.ex(e[2])
            d = "+" if e[1] == "++" else "-"
            if is_arith(t.ty):
                return [self.store(t.lv, "%s %s 1" % (t.code, d))]
            if isinstance(t.ty, PtrT) or (isinstance(t.ty, Cls) and t.ty.name == "iterator"):
                return [self.store(t.lv, "%s(%s)" % ("_inc" if d == "+" else "_dec", t.code))]
            raise Unsupported("++ on %r" % t.ty)
        if k == "assign":
            return self.assign_stmt(e)
        if k == "bin" and e[1] == "<<" and self._is_stream(e):
            return []                                   # std::cout / cerr output: no effect here
        if k == "call":
            c, pre, post = self.ex_full(e)
            return pre + [c.code] + post
        if k == "member" or k == "name":
            return []
        raise Unsupported("expression statement %s" % k)

    def assign_stmt(self, e):
        _, op, lhs_n, rhs_n = e
        if op == "=" and rhs_n[0] == "post":          # x = y++: the old value, then the increment
            return self.assign_stmt(("assign", "=", lhs_n, rhs_n[2])) + self.expr_stmt(rhs_n, 0)
        # comma on the right: the side effects in order, then the last value
        pre = []
        while rhs_n[0] == "paren":
            rhs_n = rhs_n[1]
        if rhs_n[0] == "comma":
            for x in rhs_n[1][:-1]:
                pre += self.expr_stmt(x, 0)
            rhs_n = rhs_n[1][-1]
        lhs, lpre, lpost = self.ex_full(lhs_n)
        rhs, cpre, cpost = self.ex_full(rhs_n)
        if cpost or lpost:
            raise Unsupported("out-parameters in an assignment")
        pre += lpre + cpre
        lt = lhs.ty
        if op == "=":
            if is_obj(lt):
                if isinstance(rhs.ty, Cls) and rhs.ty.name == "MatExpr":
                    return pre + ["_assign(%s, %s)" % (lhs.code, rhs.code)]
                self.conv(rhs, lt)
                return pre + ["_assign(%s, %s)" % (lhs.code, rhs.code)]
            if isinstance(lt, Prim) or isinstance(lt, PtrT) or (isinstance(lt, Cls) and lt.name == "iterator"):
                return pre + [self.store(lhs.lv, self.conv(rhs, lt))]
            if isinstance(lt, Cls) and lt.name in VALUE_CLASSES:
                return pre + [self.store(lhs.lv, self.conv(rhs, lt))]
            raise Unsupported("assignment to %r" % lt)
        bop = op[:-1]
        if is_obj(lt) and lt == Cls("Point2f") and bop == "*":
            return pre + ["_point_imul(%s, %s)" % (lhs.code, self.conv(rhs, FLOAT))]
        if isinstance(lt, PtrT) and bop in ("+", "-"):
            return pre + [self.store(lhs.lv, "(%s %s %s)" % (lhs.code, bop, self.conv(rhs, INT)))]
        if not (is_arith(lt) and is_arith(rhs.ty)):
            raise Unsupported("compound assignment %s on %r" % (op, lt))
        val = self.ex_bin(("bin", bop, ("__e", lhs), ("__e", rhs)))
        return pre + [self.store(lhs.lv, self.conv(val, lt))]

    @staticmethod
    def _is_stream(e):
        while e[0] == "bin" and e[1] == "<<":
            e = e[2]
        return e[0] == "name" and _strip(e[1]) in ("cout", "cerr", "clog")

    def ex___e(self, n):
        return n[1]

    def st_decl(self, n, ind):
        pad = "    " * ind
        lines = []
        for ty, ref, name, dims, init in n[1]:
            if dims:
                if len(dims) != 1 or init is not None:
                    raise Unsupported("array declaration %s" % name)
                d = self.conv(self.ex(dims[0]), INT)
                aty = Cls("carray", (ty,))
                py = self.declare(name, aty)
                lines.append("%s = _carray(%s, %s)" % (py, d, self.factory(ty)))
                continue
            if ref:
                if init is None or init[0] != "=":
                    raise Unsupported("reference %s without initialiser" % name)
                e, pre, post = self.ex_full(init[1])
                if post:
                    raise Unsupported("out-parameters in a reference initialiser")
                if isinstance(ty, Prim):
                    if e.lv is None:   # const T& bound to a temporary: a value
                        py = self.declare(name, ty)
                        lines += pre + ["%s = %s" % (py, self.conv(e, ty))]
                        continue
                    if e.lv[0] == "sub":
                        py = self.declare(name, ty, "cell")
                        lines += pre + ["%s = _Cell(%s, %s)" % (py, e.lv[1], e.lv[2])]
                        continue
                    py = self.declare(name, ty)     # a reference to a scalar local: alias by value
                    lines += pre + ["%s = %s" % (py, e.code)]
                    continue
                py = self.declare(name, ty, "ref")
                lines += pre + ["%s = %s" % (py, self.conv(e, ty))]
                continue
            if init is None:
                py = self.declare(name, ty)
                lines.append("%s = %s" % (py, self.default(ty)))
                continue
            if init[0] == "=":
                e, pre, post = self.ex_full(init[1])
                if post:
                    raise Unsupported("out-parameters in an initialiser")
                py = self.declare(name, ty)
                if is_obj(ty):
                    if isinstance(e.ty, Cls) and e.ty.name == "MatExpr":
                        lines += pre + ["%s = %s" % (py, self.default(ty)), "_assign(%s, %s)" % (py, e.code)]
                    else:
                        lines += pre + ["%s = _cp(%s)" % (py, self.conv(e, ty))]
                else:
                    lines += pre + ["%s = %s" % (py, self.conv(e, ty))]
                continue
            # T x(args)
            args = init[1]
            saved = self.take_prepost()
            es = [self.ex(a) for a in args]
            if self.pre or self.post:
                raise Unsupported("out-parameters in constructor arguments")
            self.pre, self.post = saved
            py = self.declare(name, ty)
            if isinstance(ty, Prim) or isinstance(ty, PtrT):
                lines.append("%s = %s" % (py, self.conv(es[0], ty)))
            elif isinstance(ty, Cls) and ty.name == "vector":
                el = ty.args[0]
                lines.append("%s = %s" % (py, self.default(ty)))
                a = [self.conv(es[0], INT)] + ([self.conv(es[1], el)] if len(es) > 1 else [])
                lines.append("%s['resize'](%s)" % (py, ", ".join(a)))
            elif isinstance(ty, Cls) and ty.name == "Vec":
                if len(es) != ty.args[1]:
                    raise Unsupported("Vec of %d with %d values" % (ty.args[1], len(es)))
                lines.append("%s = _VecInit(%s)" % (py, ", ".join(self.conv(e, ty.args[0]) for e in es)))
            else:
                spec = self.ctx.classes.get(ty.name)
                if spec is None:
                    raise Unsupported("constructor of %r" % ty)
                lines.append("%s = %s(%s)" % (py, spec.ctor, ", ".join(e.code for e in es)))
        return [pad + x for x in lines]


def translate_function(ctx, pyname, params_text, body_text, this_cls=None, ret=VOID,
                       defined=(), macros=None, init_text=None):
    """-> Python source of `def pyname([M,] params...)` for a C++ function body."""
    ft = FuncTranslator(ctx, this_cls, ret)
    pnames = []
    if params_text.strip() and params_text.strip() != "void":
        for p in split_top(params_text, ","):
            p = re.sub(r"=.*$", "", p.strip())
            toks = preprocess(p)
            ps = Parser(toks, ctx.type_names)
            r = ps.try_type()
            if r is None:
                raise Unsupported("parameter %r" % p)
            ty, ref = r
            name = ps.take().text
            is_const = p.strip().startswith("const") or " const " in p
            kind = "val"
            if ref and not is_const and isinstance(ty, Prim):
                kind = "cell"
            pnames.append(ft.declare(name, ty, kind))
    lines = []
    if init_text:
        # constructor initialiser list: member(expr), ...
        for it in split_top(init_text.strip().lstrip(":"), ","):
            m = re.fullmatch(r"\s*(\w+)\s*\((.*)\)\s*", it, re.S)
            if not m:
                raise Unsupported("initialiser %r" % it)
            mem, ex = m.group(1), m.group(2)
            lhs = ("name", mem)
            node = Parser(preprocess(ex, defined, macros), ctx.type_names).expr()
            lines += ["    " + x for x in ft.assign_stmt(("assign", "=", lhs, node))]
    toks = preprocess(body_text, defined, macros)
    body = Parser(toks, ctx.type_names).parse_body()
    lines += ft.block(body, 1)
    head = ["M"] if this_cls is not None else []
    return "def %s(%s):\n%s\n" % (pyname, ", ".join(head + pnames), "\n".join(lines))


def split_top(s, sep):
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "([<{":
            depth += 1
        elif ch in ")]>}":
            depth -= 1
        if ch == sep and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return out


def parse_members(ctx, body_text):
    """{name: Ty} of the data members declared in a class body (methods, enums, access
    specifiers and constructors skipped)."""
    out = {}
    txt = strip_comments(body_text)
    txt = re.sub(r"\b(public|private|protected)\s*:", ";", txt)
    # drop function bodies and enums
    depth, buf = 0, []
    for ch in txt:
        if ch == "{":
            depth += 1
            continue
        if ch == "}":
            depth -= 1
            buf.append(";")
            continue
        if depth == 0:
            buf.append(ch)
    for st in "".join(buf).split(";"):
        st = st.strip()
        if not st or "(" in st or st.startswith("enum") or st.startswith("typedef") or \
                st.startswith("friend") or st.startswith("using"):
            continue
        toks = preprocess(st)
        p = Parser(toks, ctx.type_names)
        r = p.try_type()
        if r is None:
            continue
        base, ref = r
        while p.i < len(p.t):
            ty = base
            while p.peek() in ("*", "&"):
                if p.take().text == "*":
                    ty = PtrT(ty)
            if p.peekk() != "id":
                break
            name = p.take().text
            out[name] = ty
            while p.i < len(p.t) and p.peek() != ",":
                p.take()
            if p.peek() == ",":
                p.take()
    return out


def make_default(ctx, ty, rt):
    """A default-constructed value of `ty` (used to build the env's element factories)."""
    if ty == INT:
        return 0
    if ty == BOOL:
        return False
    if ty in (FLOAT, DOUBLE):
        return 0.0
    if isinstance(ty, PtrT):
        return None
    if isinstance(ty, Cls):
        if ty.name == "vector":
            return rt.Vector(lambda: make_default(ctx, ty.args[0], rt))
        if ty.name == "list":
            return rt.List(lambda: make_default(ctx, ty.args[0], rt))
        if ty.name in ("map", "unordered_map"):
            return rt.Map(lambda: make_default(ctx, ty.args[1], rt), ordered=ty.name == "map")
        if ty.name == "pair":
            return rt.Pair(make_default(ctx, ty.args[0], rt), make_default(ctx, ty.args[1], rt))
        if ty.name == "iterator":
            return None
        if ty.name == "Vec":
            return rt.Vector(lambda: 0.0, [0.0] * ty.args[1])
        spec = ctx.classes.get(ty.name)
        if spec is not None and spec.fields and spec.runtime_ctor is None:
            return rt.Struct(ty.name, {k: _field_default(ctx, t, rt) for k, t in spec.fields.items()})
        if spec is not None and spec.runtime_ctor is not None:
            return spec.runtime_ctor()
    raise Unsupported("no default value for %r" % (ty,))


def _field_default(ctx, ty, rt):
    """A data member's initial value; members of classes the runtime does not model (DBoW2
    vectors, the vocabulary, ...) stay unset (None): touching one fails loudly."""
    try:
        return make_default(ctx, ty, rt)
    except Unsupported:
        return None


def build_env(ctx, rt, extra=None):
    """The env the translated functions run in: runtime helpers, factories, constants."""
    env = rt.env()
    env["_Vector"] = rt.Vector
    env["_List"] = rt.List
    env["_Map"] = lambda fac, ordered: rt.Map(fac, ordered)
    env["_carray"] = lambda n, fac: [fac() for _ in range(n)]
    env["_vector_n"] = lambda fac, n: rt.Vector(fac, [fac() for _ in range(n)])
    env["_VecN"] = lambda n: rt.Vector(lambda: 0.0, [0.0] * n)
    env["_vector_nv"] = lambda fac, n, v: rt.Vector(fac, [rt.cp(v) for _ in range(n)])
    env["_VecInit"] = lambda *xs: rt.Vector(lambda: 0.0, list(xs))
    env["_cround"] = lambda x: float(rt.c_round(x))
    for key, ty in ctx.factories.items():
        env[key] = (lambda t: (lambda: make_default(ctx, t, rt)))(ty)
    for name, spec in ctx.classes.items():
        if spec.ctor and spec.ctor not in env:
            if spec.runtime_ctor is not None:
                env[spec.ctor] = spec.runtime_ctor
            else:
                env[spec.ctor] = (lambda t: (lambda: make_default(ctx, t, rt)))(Cls(name))
    if extra:
        env.update(extra)
    return env
