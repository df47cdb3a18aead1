"""Extract the reference CLIs' argparse flags (name, type, default, action, choices)
from src/main.py and src/train_teacher_gnn.py with `ast` (the source is read as
text, nothing is imported or executed) into tests/golden/cli_flags.json, the
fixture tests/test_cli_flags.py checks the drop-in parsers against.

    python tests/golden/gen_cli_flags.py [/root/reference]
"""
import ast
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def _value(node):
    if isinstance(node, ast.Name):
        return {"int": "int", "float": "float", "str": "str"}.get(node.id, node.id)
    return ast.literal_eval(ast.unparse(node)) if not isinstance(node, ast.BinOp) else eval(
        compile(ast.Expression(node), "<flag>", "eval"), {"__builtins__": {}})


def flags(path):
    out = {}
    for node in ast.walk(ast.parse(open(path).read())):
        if not (isinstance(node, ast.Call) and isinstance(node.func, ast.Attribute)
                and node.func.attr == "add_argument"):
            continue
        name = node.args[0].value
        spec = {}
        for kw in node.keywords:
            if kw.arg in ("type", "default", "action", "choices"):
                spec[kw.arg] = _value(kw.value)
        out[name] = spec
    return out


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    res = {s: flags(os.path.join(ref, "src", s)) for s in ("main.py", "train_teacher_gnn.py")}
    with open(os.path.join(HERE, "cli_flags.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print({k: len(v) for k, v in res.items()})


if __name__ == "__main__":
    main()
