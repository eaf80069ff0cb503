"""Inert reader for the reference's waypoint files.

The reference stores each track as a pickled list ``[track_id, [x, y, z], ...]``
(read by ``splines/ParameterizedCenterline.py:93-97`` with ``pickle.load``).
We never unpickle reference files: this module walks the opcode stream with
``pickletools.genops`` (a disassembler, it executes nothing) and rebuilds the
value from the handful of inert opcodes such a list uses.  Any other opcode
(globals, reduce, build, ...) is rejected.
"""
import pickletools

_ALLOWED = {"PROTO", "FRAME", "EMPTY_LIST", "MEMOIZE", "MARK", "BININT1",
            "BININT", "BININT2", "BINFLOAT", "APPEND", "APPENDS", "STOP"}


def load_waypoint_pickle(path):
    with open(path, "rb") as f:
        data = f.read()
    stack = []
    marks = []
    result = None
    for op, arg, _pos in pickletools.genops(data):
        name = op.name
        if name not in _ALLOWED:
            raise ValueError(f"{path}: opcode {name} not allowed in a waypoint file")
        if name in ("PROTO", "FRAME", "MEMOIZE"):
            continue
        if name == "EMPTY_LIST":
            stack.append([])
        elif name == "MARK":
            marks.append(len(stack))
        elif name in ("BININT1", "BININT", "BININT2"):
            stack.append(int(arg))
        elif name == "BINFLOAT":
            stack.append(float(arg))
        elif name == "APPEND":
            v = stack.pop()
            stack[-1].append(v)
        elif name == "APPENDS":
            m = marks.pop()
            items = stack[m:]
            del stack[m:]
            stack[-1].extend(items)
        elif name == "STOP":
            result = stack.pop()
    if not isinstance(result, list):
        raise ValueError(f"{path}: not a list pickle")
    return result
