"""Reads the data of a Go table-driven test (the composite literals of its `x := ...` locals and
its `tests := []struct{...}{...}` cases) into Python values, for make_golden.py.

Only data is extracted, never code: struct literals become dicts keyed by the JSON name of each
field (ObjectMeta -> "metadata", other fields lower-camel), slice literals become lists, map
literals dicts, string / int / bool literals themselves; identifiers resolve through the test's
own locals and a table of the constants these tests use.  Run at fixture-generation time only
(against the reference checkout); the fixtures it produces are committed.
"""
import re

_TOK = re.compile(r'\s+|//[^\n]*|/\*.*?\*/|"(?:\\.|[^"\\])*"|`[^`]*`|[A-Za-z_][A-Za-z0-9_.]*|-?\d+|:=|[{}\[\]():,&*+=]',
                  re.S)

CONSTANTS = {
    "metav1.LabelSelectorOpIn": "In", "metav1.LabelSelectorOpNotIn": "NotIn",
    "metav1.LabelSelectorOpExists": "Exists", "metav1.LabelSelectorOpDoesNotExist": "DoesNotExist",
    "v1.NodeSelectorOpIn": "In", "v1.NodeSelectorOpNotIn": "NotIn", "v1.NodeSelectorOpExists": "Exists",
    "v1.NodeSelectorOpDoesNotExist": "DoesNotExist", "v1.NodeSelectorOpGt": "Gt", "v1.NodeSelectorOpLt": "Lt",
    "schedulerapi.MaxPriority": 10, "v1.DefaultHardPodAffinitySymmetricWeight": 1,
    "true": True, "false": False, "nil": None,
}
FIELD_NAMES = {"ObjectMeta": "metadata", "UID": "uid"}


def tokens(src):
    out = []
    for m in _TOK.finditer(src):
        t = m.group(0)
        if t.isspace() or t.startswith("//") or t.startswith("/*"):
            continue
        out.append(t)
    return out


def function_body(src, name):
    i = src.index("func %s(" % name)
    j = src.index("{", i)
    depth = 0
    for k in range(j, len(src)):
        if src[k] == "{":
            depth += 1
        elif src[k] == "}":
            depth -= 1
            if depth == 0:
                return src[j + 1:k]
    raise ValueError(name)


def _field(name):
    if name in FIELD_NAMES:
        return FIELD_NAMES[name]
    return name[0].lower() + name[1:]


class Parser:
    def __init__(self, toks, env, unknown=None):
        self.t, self.i, self.env = toks, 0, env
        self.unknown = unknown if unknown is not None else {}

    def peek(self, k=0):
        return self.t[self.i + k] if self.i + k < len(self.t) else None

    def take(self, want=None):
        t = self.t[self.i]
        if want is not None and t != want:
            raise ValueError("want %r got %r at %d: %s" % (want, t, self.i, " ".join(self.t[max(0, self.i - 12):self.i + 6])))
        self.i += 1
        return t

    def skip_type(self):
        """A type expression: []T, [][]T, *T, map[K]V, struct{...}, qualified ident."""
        t = self.peek()
        if t == "[":
            self.take("[")
            self.take("]")
            return self.skip_type()
        if t in ("*", "&"):
            self.take()
            return self.skip_type()
        if t == "map":
            self.take()
            self.take("[")
            self.skip_type()
            self.take("]")
            return self.skip_type()
        if t == "struct":
            self.take()
            self.take("{")
            depth = 1
            while depth:
                x = self.take()
                depth += x == "{"
                depth -= x == "}"
            return
        self.take()

    def value(self):
        v = self.unary()
        while self.peek() == "+":  # string concatenation
            self.take()
            v = v + self.unary()
        return v

    def unary(self):
        t = self.peek()
        if t == "&":
            self.take()
            return self.unary()
        if t == "{":
            return self.composite()
        if t.startswith('"'):
            self.take()
            return bytes(t[1:-1], "utf-8").decode("unicode_escape")
        if t.startswith("`"):
            self.take()
            return t[1:-1]
        if re.fullmatch(r"-?\d+", t):
            self.take()
            return int(t)
        if t in ("[", "map", "struct"):
            self.skip_type()
            return self.composite()
        # identifier: a type followed by a literal, a conversion call, or a value
        self.take()
        if self.peek() == "{" and (t[0].isupper() or "." in t):
            return self.composite()
        if self.peek() == "(":  # conversion such as int32(5) or a helper call
            self.take("(")
            args = []
            while self.peek() != ")":
                args.append(self.value())
                if self.peek() == ",":
                    self.take()
            self.take(")")
            if t in ("int32", "int64", "int", "string", "float64"):
                return args[0]
            self.unknown[t] = self.unknown.get(t, 0) + 1
            return {"__call__": t, "args": args}
        if t in self.env:
            return self.env[t]
        if t in CONSTANTS:
            return CONSTANTS[t]
        return {"__ident__": t}

    def composite(self):
        self.take("{")
        items, keyed = [], False
        while self.peek() != "}":
            if self.peek(1) == ":" and self.peek() not in ("{",):
                k = self.take()
                self.take(":")
                key = bytes(k[1:-1], "utf-8").decode("unicode_escape") if k.startswith('"') else _field(k)
                items.append((key, self.value()))
                keyed = True
            else:
                items.append(self.value())
            if self.peek() == ",":
                self.take()
        self.take("}")
        return dict(items) if keyed else items


def parse_test(src, func):
    """The locals (name := literal) of test function `func` and its `tests` case list."""
    body = tokens(function_body(src, func))
    env = {}
    p = Parser(body, env)
    cases = None
    while p.i < len(body):
        if p.peek(1) == ":=":
            name = p.take()
            p.take(":=")
            if p.peek() == "range" or p.peek() is None:
                break
            start = p.i
            try:
                val = p.value()
            except (ValueError, IndexError):
                p.i = start + 1
                continue
            if name in ("tests", "podTolerateTaintsTests", "testCases", "table"):
                cases = val
                break
            env[name] = val
        elif p.peek() == "for":
            break
        else:
            p.take()
    return env, cases
