"""The drop-in CLIs accept every flag of the reference's `main.py` /
`train_teacher_gnn.py` (src/main.py:239-269, src/train_teacher_gnn.py:271-290) with
the same type, default, action and choices; extra flags are additive only.
Fixture: tests/golden/cli_flags.json (tests/golden/gen_cli_flags.py).  CPU only."""
import argparse
import json
import os

import pytest

import main
import train_teacher_gnn

HERE = os.path.dirname(os.path.abspath(__file__))
REF = json.load(open(os.path.join(HERE, "golden", "cli_flags.json")))
PARSERS = {"main.py": main.build_parser, "train_teacher_gnn.py": train_teacher_gnn.build_parser}


def _actions(parser):
    return {s: a for a in parser._actions for s in a.option_strings}


@pytest.mark.parametrize("script", sorted(PARSERS))
def test_reference_flags_kept(script):
    acts = _actions(PARSERS[script]())
    for flag, spec in REF[script].items():
        assert flag in acts, f"{script}: {flag} missing"
        a = acts[flag]
        if spec.get("action") == "store_true":
            assert isinstance(a, argparse._StoreTrueAction), flag
            continue
        assert a.default == spec.get("default"), (flag, a.default, spec.get("default"))
        if "type" in spec:
            assert a.type is not None and a.type.__name__ == spec["type"], (flag, a.type)
        if "choices" in spec:
            assert list(a.choices) == spec["choices"], (flag, a.choices)


@pytest.mark.parametrize("script", sorted(PARSERS))
def test_reference_command_lines_parse(script):
    """A reference command line parses to the reference's values."""
    p = PARSERS[script]()
    args = p.parse_args(["--datasets", "collab", "--hidden_channels", "1024", "--num_layers", "3"])
    assert (args.datasets, args.hidden_channels, args.num_layers) == ("collab", 1024, 3)
    defaults = vars(p.parse_args([]))
    for flag, spec in REF[script].items():
        key = flag.lstrip("-")
        want = False if spec.get("action") == "store_true" else spec.get("default")
        assert defaults[key] == want, (flag, defaults[key], want)
