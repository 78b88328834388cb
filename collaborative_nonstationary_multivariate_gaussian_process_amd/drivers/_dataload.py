"""Data-only reader for the drivers' input pickles (code/NMGP_PM25.py:26-28, code/NMGP_HCP.py:24-26 read
``[X_list, Y_list, Xt_list, Yt_list]`` of numpy arrays with pickle.load).

A pickle is a program; unpickling a user's file would run whatever callables it names.  This reader
never unpickles: it walks the opcode stream with ``pickletools.genops`` (a disassembler) and interprets
the container / constant opcodes itself on a symbolic stack.  The only callables it recognises are the
numpy array and dtype constructors that numpy's own pickles name (``_reconstruct`` + BUILD state,
``_frombuffer``, ``dtype``) and ``_codecs.encode`` / ``bytes()`` (protocol-2 bytes); it evaluates them itself with
``np.frombuffer`` on the raw payload.  Any other global, object construction or out-of-band buffer
raises ``ValueError`` -- nothing from the file is ever executed.
"""
import pickletools

import numpy as np

_RECONSTRUCT = {("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct")}
_FROMBUFFER = {("numpy.core.numeric", "_frombuffer"), ("numpy._core.numeric", "_frombuffer")}
_NDARRAY = {("numpy", "ndarray")}
_DTYPE = {("numpy", "dtype")}
_ENCODE = {("_codecs", "encode")}
_BYTES = {("__builtin__", "bytes"), ("builtins", "bytes"), ("__builtin__", "bytearray"), ("builtins", "bytearray")}
_ALLOWED = _RECONSTRUCT | _FROMBUFFER | _NDARRAY | _DTYPE | _ENCODE | _BYTES


class _Global:
    def __init__(self, module, name):
        if (module, name) not in _ALLOWED:
            raise ValueError(f"refusing to load: the pickle names {module}.{name} (not numpy array data)")
        self.key = (module, name)


class _ArrayStub:            # numpy _reconstruct(ndarray, (0,), b'b') before its BUILD state
    pass


class _DtypeStub:
    def __init__(self, descr):
        self.descr = str(descr)
        self.order = "="

    def dtype(self):
        dt = np.dtype(self.descr)
        if dt.hasobject:
            raise ValueError("refusing to load: object arrays are not data")
        return dt.newbyteorder(self.order) if self.order in "<>" else dt


_MARK = object()


def _as_dtype(d):
    if isinstance(d, _DtypeStub):
        return d.dtype()
    if isinstance(d, str):
        return np.dtype(d)
    raise ValueError("refusing to load: unsupported dtype description")


def _reduce(fn, args):
    if not isinstance(fn, _Global):
        raise ValueError("refusing to load: call of a non-global")
    if fn.key in _RECONSTRUCT:
        return _ArrayStub()
    if fn.key in _DTYPE:
        return _DtypeStub(args[0])
    if fn.key in _FROMBUFFER:
        buf, dt, shape, order = args
        return np.frombuffer(bytes(buf), dtype=_as_dtype(dt)).reshape(shape, order=order).copy()
    if fn.key in _ENCODE:
        return str(args[0]).encode(args[1] if len(args) > 1 else "utf-8")
    if fn.key in _BYTES:                      # protocol 2: bytes() / bytearray() of nothing or of bytes
        if args and not isinstance(args[0], (bytes, bytearray)):
            raise ValueError("refusing to load: bytes() of a non-bytes argument")
        return bytes(args[0]) if args else b""
    raise ValueError(f"refusing to load: {fn.key}")


def _build(obj, state):
    if isinstance(obj, _DtypeStub):
        if isinstance(state, tuple) and len(state) > 1 and state[1] in ("<", ">", "|", "="):
            obj.order = state[1]
        return obj
    if isinstance(obj, _ArrayStub):
        _, shape, dt, fortran, raw = state
        if not isinstance(raw, (bytes, bytearray)):
            raise ValueError("refusing to load: array payload is not raw bytes")
        a = np.frombuffer(bytes(raw), dtype=_as_dtype(dt))
        return a.reshape(tuple(shape), order="F" if fortran else "C").copy()
    raise ValueError("refusing to load: BUILD of an object that is not numpy array data")


def load_data_pickle(path):
    """The object stored in `path` if it consists only of lists / tuples / dicts of numpy arrays, numbers,
    strings and bytes; ValueError for anything else."""
    with open(path, "rb") as fh:
        data = fh.read()
    stack, memo = [], {}

    def pop_mark():
        i = len(stack) - 1
        while stack[i] is not _MARK:
            i -= 1
        items = stack[i + 1:]
        del stack[i:]
        return items

    for op, arg, _ in pickletools.genops(data):
        n = op.name
        if n in ("PROTO", "FRAME"):
            continue
        if n == "STOP":
            break
        if n == "MARK":
            stack.append(_MARK)
        elif n in ("EMPTY_LIST",):
            stack.append([])
        elif n == "EMPTY_TUPLE":
            stack.append(())
        elif n == "EMPTY_DICT":
            stack.append({})
        elif n == "LIST":
            stack.append(list(pop_mark()))
        elif n == "TUPLE":
            stack.append(tuple(pop_mark()))
        elif n in ("TUPLE1", "TUPLE2", "TUPLE3"):
            k = int(n[-1])
            items = tuple(stack[-k:])
            del stack[-k:]
            stack.append(items)
        elif n == "DICT":
            items = pop_mark()
            stack.append({items[i]: items[i + 1] for i in range(0, len(items), 2)})
        elif n == "APPEND":
            v = stack.pop()
            stack[-1].append(v)
        elif n == "APPENDS":
            items = pop_mark()
            stack[-1].extend(items)
        elif n == "SETITEM":
            v = stack.pop()
            k = stack.pop()
            stack[-1][k] = v
        elif n == "SETITEMS":
            items = pop_mark()
            for i in range(0, len(items), 2):
                stack[-1][items[i]] = items[i + 1]
        elif n in ("BININT", "BININT1", "BININT2", "INT", "LONG", "LONG1", "LONG4", "BINFLOAT", "FLOAT",
                   "BINUNICODE", "SHORT_BINUNICODE", "BINUNICODE8", "UNICODE", "BINSTRING", "SHORT_BINSTRING",
                   "STRING", "BINBYTES", "SHORT_BINBYTES", "BINBYTES8"):
            stack.append(arg)
        elif n == "BYTEARRAY8":
            stack.append(bytearray(arg))
        elif n == "NONE":
            stack.append(None)
        elif n in ("NEWTRUE", "NEWFALSE"):
            stack.append(n == "NEWTRUE")
        elif n == "GLOBAL":
            module, name = arg.split(" ", 1)
            stack.append(_Global(module, name))
        elif n == "STACK_GLOBAL":
            name = stack.pop()
            module = stack.pop()
            stack.append(_Global(module, name))
        elif n == "REDUCE":
            args = stack.pop()
            fn = stack.pop()
            stack.append(_reduce(fn, args))
        elif n == "BUILD":
            state = stack.pop()
            stack[-1] = _build(stack[-1], state)
        elif n in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[arg] = stack[-1]
        elif n == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif n in ("BINGET", "LONG_BINGET", "GET"):
            stack.append(memo[arg])
        elif n == "POP":
            stack.pop()
        elif n == "POP_MARK":
            pop_mark()
        elif n == "DUP":
            stack.append(stack[-1])
        else:
            raise ValueError(f"refusing to load: pickle opcode {n} is not plain data")
    if len(stack) != 1:
        raise ValueError("malformed data pickle")
    out = stack[0]
    if isinstance(out, (_ArrayStub, _DtypeStub, _Global)):
        raise ValueError("malformed data pickle")
    return out
