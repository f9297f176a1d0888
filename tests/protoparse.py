"""Test infrastructure: a reader for the proto2 subset the reference's data-transfer schema uses
(src/proto/datatransfer.proto, hdfs.proto, Security.proto), producing
google.protobuf.descriptor_pb2.FileDescriptorProto objects that google.protobuf's own runtime turns
into message classes. It lets Google's encoder and decoder — not this repo's codec — produce and
check the wire bytes of every message the checksum path exchanges (tests/golden/make_proto_golden.py).

Supported: `syntax`, `package`, `import`, `option` (ignored), nested `message` / `enum`, fields
`required|optional|repeated <type> <name> = <n> [default = v, packed = b];`, // and /* */ comments.
Anything else raises, so a schema outside the subset is never half-read."""
import re

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_SCALARS = {
    "double": 1, "float": 2, "int64": 3, "uint64": 4, "int32": 5, "fixed64": 6, "fixed32": 7, "bool": 8,
    "string": 9, "bytes": 12, "uint32": 13, "sfixed32": 15, "sfixed64": 16, "sint32": 17, "sint64": 18,
}
_LABELS = {"optional": 1, "required": 2, "repeated": 3}
_TOKEN = re.compile(r'\s+|//[^\n]*|/\*.*?\*/|("(?:[^"\\]|\\.)*")|([A-Za-z_][\w.]*)|(-?\d+(?:\.\d+)?)|(\S)', re.S)


def _tokens(text):
    out = []
    for m in _TOKEN.finditer(text):
        tok = m.group(1) or m.group(2) or m.group(3) or m.group(4)
        if tok:
            out.append(tok)
    return out


class _Parser:
    def __init__(self, toks, name):
        self.t, self.i = toks, 0
        self.fd = descriptor_pb2.FileDescriptorProto(name=name, syntax="proto2")

    def peek(self):
        return self.t[self.i] if self.i < len(self.t) else None

    def take(self, want=None):
        tok = self.t[self.i]
        self.i += 1
        if want is not None and tok != want:
            raise ValueError(f"{self.fd.name}: expected {want!r}, got {tok!r} at token {self.i}")
        return tok

    def skip_statement(self):
        while self.take() != ";":
            pass

    def parse(self):
        while self.peek() is not None:
            tok = self.take()
            if tok == "syntax":
                self.skip_statement()
            elif tok == "package":
                self.fd.package = self.take()
                self.take(";")
            elif tok == "import":
                self.fd.dependency.append(self.take().strip('"'))
                self.take(";")
            elif tok == "option":
                self.skip_statement()
            elif tok == "message":
                self.message(self.fd.message_type.add())
            elif tok == "enum":
                self.enum(self.fd.enum_type.add())
            else:
                raise ValueError(f"{self.fd.name}: unsupported top-level token {tok!r}")
        return self.fd

    def enum(self, e):
        e.name = self.take()
        self.take("{")
        while self.peek() != "}":
            if self.peek() == "option":
                self.take()
                self.skip_statement()
                continue
            v = e.value.add(name=self.take())
            self.take("=")
            v.number = int(self.take())
            self.take(";")
        self.take("}")

    def message(self, m):
        m.name = self.take()
        self.take("{")
        while self.peek() != "}":
            tok = self.take()
            if tok == "message":
                self.message(m.nested_type.add())
            elif tok == "enum":
                self.enum(m.enum_type.add())
            elif tok == "option":
                self.skip_statement()
            elif tok in _LABELS:
                f = m.field.add(label=_LABELS[tok])
                typ = self.take()
                f.name = self.take()
                self.take("=")
                f.number = int(self.take())
                if typ in _SCALARS:
                    f.type = _SCALARS[typ]
                else:
                    f.type_name = typ  # resolved below: message or enum
                if self.peek() == "[":
                    self.take()
                    while True:
                        key = self.take()
                        self.take("=")
                        val = self.take()
                        if key == "default":
                            f.default_value = val.strip('"')
                        elif key == "packed":
                            f.options.packed = val == "true"
                        else:
                            raise ValueError(f"unsupported field option {key}")
                        if self.take() == "]":
                            break
                self.take(";")
            else:
                raise ValueError(f"{self.fd.name}: unsupported token {tok!r} in message {m.name}")
        self.take("}")


def _resolve(fds):
    """Fill type (11 message / 14 enum) and fully-qualified type_name for named field types,
    following protobuf's scoping: innermost enclosing scope first, then the package."""
    kinds = {}

    def collect(prefix, msgs, enums):
        for e in enums:
            kinds[f"{prefix}.{e.name}"] = 14
        for m in msgs:
            kinds[f"{prefix}.{m.name}"] = 11
            collect(f"{prefix}.{m.name}", m.nested_type, m.enum_type)

    for fd in fds:
        collect("." + fd.package, fd.message_type, fd.enum_type)

    def fix(scope, msgs):
        for m in msgs:
            inner = f"{scope}.{m.name}"
            for f in m.field:
                if f.type_name and not f.type_name.startswith("."):
                    parts = inner.split(".")
                    for k in range(len(parts), 0, -1):
                        cand = ".".join(parts[:k]) + "." + f.type_name
                        if cand in kinds:
                            f.type_name, f.type = cand, kinds[cand]
                            break
                    else:
                        raise ValueError(f"unresolved type {f.type_name} in {inner}")
            fix(inner, m.nested_type)

    for fd in fds:
        fix("." + fd.package, fd.message_type)


def load_schema(paths_by_name, extra_fields=False):
    """{'Security.proto': path, 'hdfs.proto': path, 'datatransfer.proto': path} (dependencies first)
    -> {full message name: message class} built by google.protobuf from this schema.
    extra_fields: every message gets four fields unknown to the schema (numbers 1001-1004: uint64,
    bytes, fixed32, fixed64) — serialized under this pool they are unknown fields for a decoder of
    the real schema."""
    fds = []
    for name, path in paths_by_name.items():
        with open(path) as fh:
            fds.append(_Parser(_tokens(fh.read()), name).parse())
    _resolve(fds)
    if extra_fields:
        def add(msgs):
            for m in msgs:
                for num, typ in ((1001, 4), (1002, 12), (1003, 7), (1004, 6)):
                    m.field.add(name=f"x_unknown_{num}", number=num, label=1, type=typ)
                add(m.nested_type)
        for fd in fds:
            add(fd.message_type)
    pool = descriptor_pool.DescriptorPool()
    for fd in fds:
        pool.Add(fd)
    out = {}
    for fd in fds:
        fdesc = pool.FindFileByName(fd.name)

        def walk(descs):
            for d in descs:
                out[d.full_name] = message_factory.GetMessageClass(d)
                walk(d.nested_types)

        walk(fdesc.message_types_by_name.values())
    return out
