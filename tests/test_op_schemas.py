"""Static check (CPU, no extension needed): every call of a native op
(``torch.ops.raft_stir.<op>(...)``, or ``R.<op>`` with ``R = torch.ops.raft_stir``)
in the package, the tests and the scripts matches the op's schema as declared
in ``csrc/*.cpp`` (``m.def("...")``): no more positional arguments than the
schema has, every keyword is a schema argument, every argument without a
default is supplied.  A schema change that leaves a caller behind otherwise
only shows up on the GPU box."""
import ast
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "raft_stir_amd", "csrc")


def _schemas():
    out = {}
    for f in sorted(os.listdir(CSRC)):
        if not f.endswith(".cpp"):
            continue
        src = open(os.path.join(CSRC, f)).read()
        for m in re.finditer(r'm\.def\(((?:\s*"(?:[^"\\]|\\.)*")+)\s*(?:,\s*&\w+\s*)?\)', src):
            text = "".join(re.findall(r'"((?:[^"\\]|\\.)*)"', m.group(1)))
            name, args = re.match(r"(\w+)\((.*)\)\s*->", text).groups()
            params = []
            depth, cur = 0, ""
            for ch in args:  # split on top-level commas
                if ch in "([":
                    depth += 1
                elif ch in ")]":
                    depth -= 1
                if ch == "," and depth == 0:
                    params.append(cur.strip())
                    cur = ""
                else:
                    cur += ch
            if cur.strip():
                params.append(cur.strip())
            parsed = []
            for p in params:
                decl, _, default = p.partition("=")
                parsed.append((decl.split()[-1], bool(default)))
            out[name] = parsed
    return out


def _py_files():
    for sub in ("raft_stir_amd", "tests", "scripts"):
        for d, _, fs in os.walk(os.path.join(ROOT, sub)):
            for f in fs:
                if f.endswith(".py"):
                    yield os.path.join(d, f)
    for f in ("bench.py", "__graft_entry__.py"):
        yield os.path.join(ROOT, f)


def _is_ops_ns(node):
    return (isinstance(node, ast.Attribute) and node.attr == "raft_stir" and isinstance(node.value, ast.Attribute)
            and node.value.attr == "ops")


def _calls():
    for path in _py_files():
        tree = ast.parse(open(path).read(), path)
        aliases = set()
        for node in ast.walk(tree):
            if isinstance(node, ast.Assign) and _is_ops_ns(node.value):
                aliases.update(t.id for t in node.targets if isinstance(t, ast.Name))
        for node in ast.walk(tree):
            if not isinstance(node, ast.Call) or not isinstance(node.func, ast.Attribute):
                continue
            base = node.func.value
            if _is_ops_ns(base) or (isinstance(base, ast.Name) and base.id in aliases):
                yield os.path.relpath(path, ROOT), node.lineno, node.func.attr, node


def test_schemas_parse():
    s = _schemas()
    assert len(s) > 30 and "conv_fused" in s and "corr_otf_backward" in s


def test_native_op_calls_match_schemas():
    schemas = _schemas()
    bad, n = [], 0
    for path, line, op, call in _calls():
        if op not in schemas:
            if op in ("default", "load_library"):
                continue
            bad.append(f"{path}:{line}: unknown op {op}")
            continue
        n += 1
        params = schemas[op]
        names = [p for p, _ in params]
        if any(isinstance(a, ast.Starred) for a in call.args) or any(k.arg is None for k in call.keywords):
            continue  # *args / **kwargs: not checkable statically
        npos = len(call.args)
        if npos > len(params):
            bad.append(f"{path}:{line}: {op} takes {len(params)} arguments, {npos} given")
            continue
        kw = [k.arg for k in call.keywords]
        for k in kw:
            if k not in names:
                bad.append(f"{path}:{line}: {op} has no argument '{k}'")
        for i, (p, has_default) in enumerate(params):
            if i >= npos and p not in kw and not has_default:
                bad.append(f"{path}:{line}: {op} is missing '{p}'")
    assert n > 50, n
    assert not bad, "\n".join(bad)


if __name__ == "__main__":
    pytest.main([__file__, "-q"])
