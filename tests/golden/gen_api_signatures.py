"""Extract the constructor signatures (parameter names and literal defaults) of the
reference's model classes from src/models.py and src/sageconv_updated.py with `ast`
(read as text; nothing imported or executed) into tests/golden/api_signatures.json,
the fixture tests/test_api_surface.py checks the drop-in classes against.

    python tests/golden/gen_api_signatures.py [/root/reference]
"""
import ast
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CLASSES = {"models.py": ("MLP", "GCN", "SAGE", "LinkPredictor"), "sageconv_updated.py": ("SAGEConv_updated",)}


def signatures(path, names):
    out = {}
    for node in ast.walk(ast.parse(open(path).read())):
        if not (isinstance(node, ast.ClassDef) and node.name in names):
            continue
        init = next(f for f in node.body if isinstance(f, ast.FunctionDef) and f.name == "__init__")
        args = init.args.args[1:]                       # without self
        defaults = [None] * (len(args) - len(init.args.defaults)) + list(init.args.defaults)
        params = []
        for a, d in zip(args, defaults):
            p = {"name": a.arg}
            if d is not None:
                p["default"] = ast.literal_eval(d)
            params.append(p)
        out[node.name] = {"params": params, "kwargs": init.args.kwarg is not None}
    return out


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    res = {}
    for f, names in CLASSES.items():
        res.update(signatures(os.path.join(ref, "src", f), names))
    with open(os.path.join(HERE, "api_signatures.json"), "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    print(sorted(res))


if __name__ == "__main__":
    main()
