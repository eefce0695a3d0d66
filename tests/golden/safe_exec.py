"""Checked execution of Python that the golden generators translate from the reference text.

The generators (gen_refmath.py, gen_mcsjacs1.py, gen_g2o_solver.py) cut function bodies out of
the reference checkout -- untrusted input -- and rewrite them into Python.  Before anything
runs, the translated source is parsed with `ast` and rejected unless every node is on a small
whitelist: numbers / strings / None / bools, names (no dunder names), arithmetic, comparison
and boolean operators, subscripts, tuples / dicts, assignments, `if`, `while` / `break`, `for ... in range(...)`,
`def` / `return`, and calls whose target is a plain name or one of a few whitelisted attributes
(`Matx.make`, `.t()`, `math.sqrt`, ...).  The code then runs with an empty `__builtins__`, so
a name resolves only to what the generator put in the environment.  A crafted statement such
as `double a = __import__('os').system(...)` fails the check (dunder name) and, even if it did
not, would find no `__import__` to call.
"""
import ast

_NODES = (
    ast.Module, ast.Expression, ast.FunctionDef, ast.arguments, ast.arg, ast.Return,
    ast.Assign, ast.AugAssign, ast.If, ast.For, ast.While, ast.Break, ast.Pass, ast.Expr,
    ast.Name, ast.Load, ast.Store, ast.Constant, ast.Tuple, ast.List, ast.Dict,
    ast.Subscript, ast.Slice,
    ast.Call, ast.Attribute,
    ast.BinOp, ast.UnaryOp, ast.BoolOp, ast.Compare, ast.IfExp,
    ast.Add, ast.Sub, ast.Mult, ast.Div, ast.Mod, ast.Pow, ast.USub, ast.UAdd, ast.Not,
    ast.And, ast.Or, ast.Eq, ast.NotEq, ast.Lt, ast.LtE, ast.Gt, ast.GtE,
    # cxx_eval.py (round 5): loops with continue, bit operators, pointer null tests
    ast.Continue, ast.BitAnd, ast.BitOr, ast.BitXor, ast.LShift, ast.RShift, ast.Invert,
    ast.Is, ast.IsNot,
)
_ATTRS = {"make", "eye", "t", "get_minor", "sqrt", "atan", "pow", "fabs", "log"}


class UnsafeSource(ValueError):
    pass


def check(src, mode="exec"):
    """Parse `src` and return its AST if every node is whitelisted, else raise UnsafeSource."""
    tree = ast.parse(src, mode=mode)
    for node in ast.walk(tree):
        if not isinstance(node, _NODES):
            raise UnsafeSource("node %s not allowed in translated reference code" % type(node).__name__)
        if isinstance(node, ast.Name) and node.id.startswith("__"):
            raise UnsafeSource("dunder name %r in translated reference code" % node.id)
        if isinstance(node, ast.Attribute) and (node.attr not in _ATTRS or node.attr.startswith("_")):
            raise UnsafeSource("attribute %r not allowed in translated reference code" % node.attr)
        if isinstance(node, ast.Constant) and not isinstance(node.value, (int, float, bool, str, type(None))):
            raise UnsafeSource("constant %r not allowed" % (node.value,))
        if isinstance(node, ast.Call) and not isinstance(node.func, (ast.Name, ast.Attribute, ast.Subscript)):
            raise UnsafeSource("call target must be a name, a whitelisted attribute or a subscript")
        if isinstance(node, ast.For):
            it = node.iter
            if not (isinstance(it, ast.Call) and isinstance(it.func, ast.Name) and it.func.id == "range"):
                raise UnsafeSource("for loops must iterate over range(...)")
    return tree


def safe_exec(src, env, filename):
    """Check `src`, then execute it with no builtins in a copy of `env`; returns the globals."""
    tree = check(src, "exec")
    g = dict(env)
    g["__builtins__"] = {}
    exec(compile(tree, filename, "exec"), g)
    return g


def safe_compile_eval(expr, filename):
    """Check an expression and compile it for `safe_eval`."""
    return compile(check(expr, "eval"), filename, "eval")


def safe_eval(code, env):
    g = dict(env)
    g["__builtins__"] = {}
    return eval(code, g)
