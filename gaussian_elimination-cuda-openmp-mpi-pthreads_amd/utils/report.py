"""Machine-readable result lines (one JSON object per line) — the reference
only printed free text that was copied into PDFs by hand."""
from __future__ import annotations

import json
import math
import sys


def _clean(v):
    if isinstance(v, float) and (math.isnan(v) or math.isinf(v)):
        return None
    if isinstance(v, dict):
        return {k: _clean(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_clean(x) for x in v]
    return v


def json_line(obj: dict, file=None) -> str:
    s = json.dumps(_clean(obj), sort_keys=False)
    print(s, file=file or sys.stdout, flush=True)
    return s
