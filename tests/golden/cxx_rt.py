"""Runtime of the Python that tests/golden/cxx_eval.py translates from the reference's C++ text.

The translated code runs under safe_exec (AST whitelist, no builtins); everything it can name
comes from `env()` below: C numeric conversions, the standard containers the reference uses
(std::vector, std::list with stable iterators, std::pair), pointers, and value semantics for
classes (copy on declaration / push, in-place assignment).  Test infrastructure only: the
golden generators use it to evaluate the reference text; nothing here is the product.

Conventions
  * a class object is a `Struct` (fields by name: obj['f']); methods of translated classes are
    free functions taking the object first; runtime classes (Vector, List, Mat, ...) answer
    obj['method'] with a bound method;
  * `Ptr(obj)` points at an object, `Ptr(seq, i)` at element i of a sequence (pointer
    arithmetic moves i); ordering of pointers (std::sort of (size, Node*) pairs) compares the
    pointee's allocation serial -- every Struct gets the next serial when it is constructed
    or copied, i.e. the addresses of a monotone allocator;
  * iterators and pointers are immutable values (`++it` rebinds), class objects are mutable.
"""
import math
import struct

import numpy as np

_serial = [0]


def _next_serial():
    _serial[0] += 1
    return _serial[0]


# ------------------------------------------------------------------ C numeric conversions
_F = struct.Struct("f")


def f32(x):
    """Round a double to float (C's double -> float conversion, round to nearest even)."""
    try:
        return _F.unpack(_F.pack(x))[0]
    except OverflowError:
        return math.copysign(math.inf, x)


def trunc(x):
    """C's floating -> integer conversion (toward zero); integers and bools unchanged."""
    if isinstance(x, float):
        if x != x or x in (math.inf, -math.inf):
            raise ValueError("undefined float -> int conversion of %r" % x)
        return int(x)
    return int(x)


def dbl(x):
    return float(x)


def idiv(a, b):
    """C integer division (truncation toward zero)."""
    a, b = int(a), int(b)
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def imod(a, b):
    a, b = int(a), int(b)
    return a - idiv(a, b) * b


def cv_round(x):
    """cvRound: _mm_cvtsd_si32 / _mm_cvtss_si32 under the default rounding mode (to nearest even)."""
    return int(round(x)) if isinstance(x, float) else int(x)


def c_round(x):
    """C round(): half away from zero."""
    return math.floor(x + 0.5) if x >= 0 else -math.floor(-x + 0.5)


def cv_floor(x):
    return int(math.floor(x))


def cv_ceil(x):
    return int(math.ceil(x))


def std_max(a, b):
    return b if a < b else a


def std_min(a, b):
    return b if b < a else a


def popcount64(x):
    return bin(int(x) & 0xFFFFFFFFFFFFFFFF).count("1")


def lt(a, b):
    """C++ operator< of the values std::sort compares (numbers, pairs, pointers)."""
    if isinstance(a, Pair):
        if lt(a.f["first"], b.f["first"]):
            return True
        if lt(b.f["first"], a.f["first"]):
            return False
        return lt(a.f["second"], b.f["second"])
    if isinstance(a, Ptr):
        return a.address() < b.address()
    return a < b


class _Key:
    __slots__ = ("v",)

    def __init__(self, v):
        self.v = v

    def __lt__(self, o):
        return lt(self.v, o.v)


# ------------------------------------------------------------------ objects
class Struct:
    """A class object: fields by name, allocation serial, optional per-field C conversions."""
    __slots__ = ("f", "serial", "cls")

    def __init__(self, cls, fields):
        self.cls = cls
        self.f = fields
        self.serial = _next_serial()

    def __getitem__(self, k):
        return self.f[k]

    def __setitem__(self, k, v):
        self.f[k] = v

    def copy(self):
        return Struct(self.cls, {k: cp(v) for k, v in self.f.items()})

    def assign(self, o):
        for k, v in o.f.items():
            cur = self.f.get(k)
            if _mutable(cur):
                assign(cur, v)
            else:
                self.f[k] = cp(v)


def _mutable(x):
    return isinstance(x, (Struct, Vector, List, Mat, Pair, Map))


def cp(x):
    """Value copy (C++ copy construction)."""
    if _mutable(x):
        return x.copy()
    return x


def assign(dst, src):
    """In-place C++ copy assignment of a class object."""
    if isinstance(src, MatExpr):
        src.assign_to(dst)
        return dst
    dst.assign(src)
    return dst


class Pair:
    __slots__ = ("f",)

    def __init__(self, a=None, b=None):
        self.f = {"first": a, "second": b}

    def __getitem__(self, k):
        return self.f[k]

    def __setitem__(self, k, v):
        self.f[k] = v

    def copy(self):
        return Pair(cp(self.f["first"]), cp(self.f["second"]))

    def assign(self, o):
        self.f["first"] = cp(o.f["first"])
        self.f["second"] = cp(o.f["second"])


class Ptr:
    """Pointer: to an object (seq None) or to element `i` of a sequence (list / Vector /
    numpy array / Mat buffer)."""
    __slots__ = ("seq", "i", "obj")

    def __init__(self, seq=None, i=0, obj=None):
        self.seq, self.i, self.obj = seq, i, obj

    def deref(self):
        if self.seq is None:
            return self.obj
        return _seq_get(self.seq, self.i)

    def __getitem__(self, k):
        if isinstance(k, str):
            return self.deref()[k]
        return _seq_get(self.seq, self.i + k)

    def __setitem__(self, k, v):
        if isinstance(k, str):
            self.deref()[k] = v
        else:
            _seq_set(self.seq, self.i + k, v)

    def __add__(self, k):
        if self.seq is None:
            raise ValueError("arithmetic on an object pointer")
        return Ptr(self.seq, self.i + int(k))

    def __sub__(self, k):
        if isinstance(k, Ptr):
            return self.i - k.i
        return Ptr(self.seq, self.i - int(k))

    def __eq__(self, o):
        if o is None:
            return False
        return isinstance(o, Ptr) and self.seq is o.seq and self.i == o.i and self.obj is o.obj

    def __ne__(self, o):
        return not self.__eq__(o)

    def __hash__(self):
        return hash((id(self.seq), self.i, id(self.obj)))

    def __bool__(self):
        return True

    def __lt__(self, o):
        return self.address() < o.address()

    def address(self):
        if self.seq is None:
            return (self.obj.serial, 0)
        return (id(self.seq), self.i)


def _seq_get(seq, i):
    if i < 0:
        raise IndexError("negative element index %d" % i)
    if isinstance(seq, Vector):
        return seq.v[i]
    v = seq[i]
    if isinstance(v, np.integer):       # a Mat byte reads as a C int (integral promotion)
        return int(v)
    return v


def _seq_set(seq, i, v):
    if i < 0:
        raise IndexError("negative element index %d" % i)
    if isinstance(seq, Vector):
        seq.v[i] = v
    else:
        seq[i] = v


class PointView:
    """`(const Point*)int_array`: the int array read as consecutive (x, y) points."""

    def __init__(self, arr):
        self.arr = arr

    def __getitem__(self, i):
        return Point2i(self.arr[2 * i], self.arr[2 * i + 1])


class Cell:
    """A reference to a scalar lvalue (container[key]), read and written as cell[0]."""
    __slots__ = ("c", "k")

    def __init__(self, c, k):
        self.c, self.k = c, k

    def __getitem__(self, i):
        return self.c[self.k]

    def __setitem__(self, i, v):
        self.c[self.k] = v


# ------------------------------------------------------------------ std::vector
class VecIt:
    __slots__ = ("vec", "i")

    def __init__(self, vec, i):
        self.vec, self.i = vec, i

    def __eq__(self, o):
        return isinstance(o, VecIt) and o.vec is self.vec and o.i == self.i

    def __ne__(self, o):
        return not self.__eq__(o)

    def __add__(self, k):
        return VecIt(self.vec, self.i + int(k))

    def __sub__(self, o):
        if isinstance(o, VecIt):
            return self.i - o.i
        return VecIt(self.vec, self.i - int(o))

    def deref(self):
        return self.vec.v[self.i]

    def __getitem__(self, k):
        return self.deref()[k]

    def __setitem__(self, k, v):
        self.deref()[k] = v

    def inc(self):
        return VecIt(self.vec, self.i + 1)

    def dec(self):
        return VecIt(self.vec, self.i - 1)


class Vector:
    __slots__ = ("v", "fac")

    def __init__(self, fac, items=None):
        self.fac = fac                  # default element
        self.v = items if items is not None else []

    def copy(self):
        return Vector(self.fac, [cp(x) for x in self.v])

    def assign(self, o):
        self.v = [cp(x) for x in o.v]

    # element access (operator[] with C's integer index conversion done by the translator)
    def __getitem__(self, k):
        if isinstance(k, str):
            return getattr(self, "m_" + k)
        if k < 0:
            raise IndexError("vector index %d" % k)
        return self.v[k]

    def __setitem__(self, k, val):
        if k < 0:
            raise IndexError("vector index %d" % k)
        self.v[k] = val

    def m_size(self):
        return len(self.v)

    def m_empty(self):
        return len(self.v) == 0

    def m_reserve(self, n):
        return None

    def m_resize(self, n, val=None):
        n = int(n)
        if n < len(self.v):
            del self.v[n:]
        while len(self.v) < n:
            self.v.append(self.fac() if val is None else cp(val))

    def m_clear(self):
        self.v = []

    def m_push_back(self, x):
        self.v.append(cp(x))

    def m_pop_back(self):
        self.v.pop()

    def m_front(self):
        return self.v[0]

    def m_back(self):
        return self.v[-1]

    def m_begin(self):
        return VecIt(self, 0)

    def m_end(self):
        return VecIt(self, len(self.v))

    def m_erase(self, first, last=None):
        if last is None:
            del self.v[first.i]
            return VecIt(self, first.i)
        del self.v[first.i:last.i]
        return VecIt(self, first.i)

    def m_insert(self, pos, first, last=None):
        if last is None:
            self.v.insert(pos.i, cp(first))
            return
        items = [cp(first.vec.v[i]) for i in range(first.i, last.i)]
        self.v[pos.i:pos.i] = items

    def m_data(self):
        return Ptr(self, 0)


# ------------------------------------------------------------------ std::list
class _Node:
    __slots__ = ("prev", "next", "val")

    def __init__(self, val):
        self.prev = self.next = None
        self.val = val


class ListIt:
    __slots__ = ("lst", "node")

    def __init__(self, lst, node):
        self.lst, self.node = lst, node

    def __eq__(self, o):
        return isinstance(o, ListIt) and o.node is self.node

    def __ne__(self, o):
        return not self.__eq__(o)

    def deref(self):
        if self.node is self.lst.head:
            raise IndexError("dereference of list end()")
        return self.node.val

    def __getitem__(self, k):
        return self.deref()[k]

    def __setitem__(self, k, v):
        self.deref()[k] = v

    def inc(self):
        return ListIt(self.lst, self.node.next)

    def dec(self):
        return ListIt(self.lst, self.node.prev)


class List:
    """std::list: a doubly linked ring with a sentinel; iterators stay valid until erased."""
    __slots__ = ("head", "n", "fac")

    def __init__(self, fac):
        self.fac = fac
        self.head = _Node(None)
        self.head.prev = self.head.next = self.head
        self.n = 0

    def __getitem__(self, k):
        return getattr(self, "m_" + k)

    def _link_before(self, node, val):
        nd = _Node(val)
        nd.prev, nd.next = node.prev, node
        node.prev.next = nd
        node.prev = nd
        self.n += 1
        return nd

    def copy(self):
        out = List(self.fac)
        nd = self.head.next
        while nd is not self.head:
            out._link_before(out.head, cp(nd.val))
            nd = nd.next
        return out

    def m_size(self):
        return self.n

    def m_empty(self):
        return self.n == 0

    def m_push_back(self, x):
        self._link_before(self.head, cp(x))

    def m_push_front(self, x):
        self._link_before(self.head.next, cp(x))

    def m_front(self):
        return self.head.next.val

    def m_back(self):
        return self.head.prev.val

    def m_begin(self):
        return ListIt(self, self.head.next)

    def m_end(self):
        return ListIt(self, self.head)

    def m_erase(self, it):
        nd = it.node
        if nd is self.head:
            raise IndexError("erase(end())")
        nd.prev.next = nd.next
        nd.next.prev = nd.prev
        self.n -= 1
        nxt = nd.next
        nd.prev = nd.next = None      # a later use of the erased iterator fails loudly
        return ListIt(self, nxt)

    def m_clear(self):
        self.head.prev = self.head.next = self.head
        self.n = 0


# ------------------------------------------------------------------ std::map / unordered_map
class MapIt:
    __slots__ = ("m", "k")

    def __init__(self, m, k):
        self.m, self.k = m, k

    def __eq__(self, o):
        return isinstance(o, MapIt) and o.m is self.m and o.k == self.k

    def __ne__(self, o):
        return not self.__eq__(o)

    def deref(self):
        if self.k is _END:
            raise IndexError("dereference of map end()")
        return self.m.pair(self.k)

    def __getitem__(self, k):
        return self.deref()[k]

    def inc(self):
        keys = self.m.keys()
        i = keys.index(self.k)
        return MapIt(self.m, keys[i + 1] if i + 1 < len(keys) else _END)


_END = object()


class _MapPair(Pair):
    """The (key, value) of a map element; writing .second writes the map."""
    __slots__ = ("m",)

    def __init__(self, m, k):
        Pair.__init__(self, k, m.d[k])
        self.m = m

    def __setitem__(self, k, v):
        if k != "second":
            raise ValueError("map keys are const")
        self.m.d[self.f["first"]] = v
        self.f["second"] = v


class Map:
    """std::map (ordered by key) / std::unordered_map (iteration order is not used by the
    translated code: find / operator[] / count only)."""
    __slots__ = ("d", "fac", "ordered")

    def __init__(self, fac, ordered=False):
        self.d, self.fac, self.ordered = {}, fac, ordered

    def copy(self):
        m = Map(self.fac, self.ordered)
        m.d = {k: cp(v) for k, v in self.d.items()}
        return m

    def assign(self, o):
        self.d = {k: cp(v) for k, v in o.d.items()}

    def keys(self):
        if not self.ordered:
            raise ValueError("iteration over an unordered_map (order unspecified)")
        return sorted(self.d)

    def pair(self, k):
        return _MapPair(self, k)

    def __getitem__(self, k):
        if isinstance(k, str) and k in ("find", "count", "begin", "end", "size", "empty", "clear"):
            return getattr(self, "m_" + k)
        if k not in self.d:
            self.d[k] = self.fac()
        return self.d[k]

    def __setitem__(self, k, v):
        self.d[k] = v

    def m_clear(self):
        self.d = {}

    def m_find(self, k):
        return MapIt(self, k if k in self.d else _END)

    def m_count(self, k):
        return 1 if k in self.d else 0

    def m_begin(self):
        ks = self.keys()
        return MapIt(self, ks[0] if ks else _END)

    def m_end(self):
        return MapIt(self, _END)

    def m_size(self):
        return len(self.d)

    def m_empty(self):
        return not self.d


def deref(p):
    if isinstance(p, (Ptr, VecIt, ListIt, MapIt)):
        return p.deref()
    if p is None:
        raise ValueError("null pointer dereference")
    return p                            # smart pointers / references to objects


def inc(it):
    if isinstance(it, Ptr):
        return it + 1
    return it.inc()


def dec(it):
    if isinstance(it, Ptr):
        return it - 1
    return it.dec()


def addr(obj):
    if obj is None:
        raise ValueError("address of nothing")
    return Ptr(obj=obj)


def addr_elem(seq, i):
    return Ptr(seq, int(i))


def std_sort(first, last):
    if isinstance(first, VecIt):
        vec = first.vec
        seg = vec.v[first.i:last.i]
        seg.sort(key=_Key)              # strict weak order of distinct keys: the unique result
        vec.v[first.i:last.i] = seg
        return
    raise ValueError("sort over %r" % (first,))


def std_remove(first, last, value):
    """std::remove on a vector range: keeps the other elements in order, returns the new end."""
    vec = first.vec
    seg = vec.v[first.i:last.i]
    kept = [x for x in seg if not (x == value)]
    vec.v[first.i:first.i + len(kept)] = kept
    return VecIt(vec, first.i + len(kept))


def std_copy(first, last, out):
    i = first.i
    while i < last.i:
        out(first.seq[i] if not isinstance(first.seq, Vector) else first.seq.v[i])
        i += 1


def back_inserter(vec):
    return vec.m_push_back


# ------------------------------------------------------------------ small OpenCV value types
def _struct(cls, **fields):
    return Struct(cls, fields)


def Point2i(x=0, y=0):
    return _struct("Point2i", x=trunc(x), y=trunc(y))


def Point2f(x=0.0, y=0.0):
    return _struct("Point2f", x=f32(x), y=f32(y))


def Point2d(x=0.0, y=0.0):
    return _struct("Point2d", x=dbl(x), y=dbl(y))


def point2d_from_vec(v):
    """cv::Point_<double>(const Vec<double, 2>& v): (v[0], v[1])."""
    return Point2d(v.v[0], v.v[1])


def KeyPoint():
    return _struct("KeyPoint", pt=Point2f(), size=0.0, angle=-1.0, response=0.0, octave=0, class_id=-1)


def Size(w=0, h=0):
    return _struct("Size", width=trunc(w), height=trunc(h))


def Rect(x=0, y=0, w=0, h=0):
    return _struct("Rect", x=trunc(x), y=trunc(y), width=trunc(w), height=trunc(h))


def Vec(n, fac=0.0):
    return Vector(lambda: fac, [fac] * n)


def point_imul(p, s):
    """Point2f *= float (cv::Point_ operator*=, the product rounded to float)."""
    p["x"] = f32(p["x"] * s)
    p["y"] = f32(p["y"] * s)
    return p


# ------------------------------------------------------------------ cv::Mat (8-bit, 2D)
class Mat:
    """A cv::Mat header: a view (r0, c0, rows, cols) into a shared 2D uint8 buffer."""
    __slots__ = ("buf", "r0", "c0", "rows", "cols")

    def __init__(self, buf=None, r0=0, c0=0, rows=None, cols=None):
        self.buf = buf
        self.r0, self.c0 = r0, c0
        self.rows = (buf.shape[0] if buf is not None else 0) if rows is None else rows
        self.cols = (buf.shape[1] if buf is not None else 0) if cols is None else cols

    def __getitem__(self, k):
        if k in ("rows", "cols"):
            return getattr(self, k)
        return getattr(self, "m_" + k)

    def copy(self):                     # copying a header shares the data
        return Mat(self.buf, self.r0, self.c0, self.rows, self.cols)

    def assign(self, o):
        self.buf, self.r0, self.c0, self.rows, self.cols = o.buf, o.r0, o.c0, o.rows, o.cols

    def view(self):
        if self.buf is None:
            return np.zeros((0, 0), np.uint8)
        return self.buf[self.r0:self.r0 + self.rows, self.c0:self.c0 + self.cols]

    def m_empty(self):
        return self.buf is None or self.rows * self.cols == 0

    def m_type(self):
        return 0                         # CV_8UC1

    def m_depth(self):
        return 0                         # CV_8U

    def m_step1(self):
        return self.buf.shape[1]

    def _range_check(self, a, b, n):
        if self.buf is None:
            raise ValueError("rowRange / colRange of an empty Mat (cv::Mat asserts dims >= 2)")
        if not (0 <= a <= b <= n):
            raise ValueError("Mat range [%d, %d) outside [0, %d)" % (a, b, n))

    def m_rowRange(self, a, b):
        self._range_check(a, b, self.rows)
        return Mat(self.buf, self.r0 + a, self.c0, b - a, self.cols)

    def m_colRange(self, a, b):
        self._range_check(a, b, self.cols)
        return Mat(self.buf, self.r0, self.c0 + a, self.rows, b - a)

    def m_call(self, rect):              # Mat::operator()(Rect)
        x, y, w, h = rect["x"], rect["y"], rect["width"], rect["height"]
        if not (0 <= x and 0 <= y and x + w <= self.cols and y + h <= self.rows):
            raise ValueError("ROI outside the Mat")
        return Mat(self.buf, self.r0 + y, self.c0 + x, h, w)

    def m_ptr(self, row):
        return Ptr(self.buf.reshape(-1), (self.r0 + row) * self.buf.shape[1] + self.c0)

    def m_ptr_uint64_t(self, row):
        """ptr<uint64_t>(row) of a byte matrix whose rows are whole 64-bit words."""
        if self.cols % 8:
            raise ValueError("ptr<uint64_t> of a row of %d bytes" % self.cols)
        words = np.ascontiguousarray(self.view()).view("<u8").reshape(-1)
        return Ptr(words, row * (self.cols // 8))

    def m_at(self, r, c=None):
        if c is None:
            return int(self.view().reshape(-1)[r])
        return int(self.buf[self.r0 + r, self.c0 + c])

    def m_addr_at(self, r, c):
        return Ptr(self.buf.reshape(-1), (self.r0 + r) * self.buf.shape[1] + self.c0 + c)

    def create(self, rows, cols):
        """Mat::create: reallocates only when the size differs (a view keeps its data)."""
        if self.buf is not None and self.rows == rows and self.cols == cols:
            return
        self.buf = np.zeros((rows, cols), np.uint8)
        self.r0 = self.c0 = 0
        self.rows, self.cols = rows, cols


class MatExpr:
    """Mat::zeros(rows, cols, type): assigning it create()s the destination, then zeroes it
    (MatOp_Initializer::assign), so a destination view of the right size stays a view."""

    def __init__(self, rows, cols):
        self.rows, self.cols = rows, cols

    def assign_to(self, m):
        m.create(self.rows, self.cols)
        m.view()[...] = 0


def mat_zeros(rows, cols, typ):
    return MatExpr(int(rows), int(cols))


def mat_new(size=None, typ=0):
    if size is None:
        return Mat()
    return Mat(np.zeros((size["height"], size["width"]), np.uint8))


class InputArray:
    def __init__(self, mat):
        self.mat = mat

    def __getitem__(self, k):
        return getattr(self, "m_" + k)

    def m_empty(self):
        return self.mat.m_empty()

    def m_getMat(self):
        return self.mat.copy()


class OutputArray:
    def __init__(self):
        self.mat = Mat()

    def __getitem__(self, k):
        return getattr(self, "m_" + k)

    def m_release(self):
        self.mat = Mat()

    def m_create(self, rows, cols, typ):
        self.mat.create(int(rows), int(cols))

    def m_getMat(self):
        return self.mat.copy()


def env():
    """The names translated code may use (besides what a generator adds)."""
    return {
        "_f32": f32, "_trunc": trunc, "_dbl": dbl, "_idiv": idiv, "_imod": imod,
        "_cvRound": cv_round, "_cvFloor": cv_floor, "_cvCeil": cv_ceil,
        "_max": std_max, "_min": std_min, "_popc": popcount64,
        "_sqrt": math.sqrt, "_ceil": math.ceil, "_floor": math.floor, "_fabs": math.fabs,
        "_pow": math.pow, "_cos": math.cos, "_sin": math.sin, "_atan": math.atan,
        "_atan2": math.atan2, "_exp": math.exp, "_log": math.log,
        "_cp": cp, "_assign": assign, "_deref": deref, "_inc": inc, "_dec": dec,
        "_addr": addr, "_addr_elem": addr_elem, "_Pair": Pair, "_Cell": Cell,
        "_sort": std_sort, "_copy": std_copy, "_back_inserter": back_inserter, "_remove": std_remove,
        "_point_imul": point_imul, "_PointView": PointView, "_Point2d_vec": point2d_from_vec,
        "_range": range, "_len": len,
    }
