"""logger.py prints exactly what the reference's src/logger.py prints
(fixture tests/golden/logger_output.json, made by gen_golden.run_logger_case)."""
import contextlib
import io
import json
import os

import logger

HERE = os.path.dirname(os.path.abspath(__file__))


def test_logger_output_is_byte_identical():
    with open(os.path.join(HERE, "golden", "logger_output.json")) as f:
        cases = json.load(f)
    for c in cases:
        L = getattr(logger, c["cls"])(len(c["table"]))
        for run, rows in enumerate(c["table"]):
            for r in rows:
                L.add_result(run, tuple(r))
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            L.print_statistics(1)
            L.print_statistics()
        assert buf.getvalue() == c["stdout"], c["cls"]
