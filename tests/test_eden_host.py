"""CPU: the EDEN sign-table cache (eden._SignCache, host logic) is bounded by bytes, evicts the
least recently used table first and always keeps the newest one."""
import torch

import uqdme  # noqa: F401
from uqdme_amd.eden import _SignCache


def test_sign_cache_byte_budget_lru():
    c = _SignCache(budget_bytes=3000, max_rows=2)
    a, b, d = (torch.zeros(1000, dtype=torch.int8) for _ in range(3))
    c.put("a", a)
    c.put("b", b)
    c.put("d", d)
    assert c.bytes == 3000 and c.get("a") is a          # "a" becomes the most recent
    c.put("e", torch.zeros(1000, dtype=torch.int8))
    assert c.get("b") is None and c.get("a") is a and c.bytes == 3000
    big = torch.zeros(10000, dtype=torch.int8)          # larger than the budget: kept alone
    c.put("big", big)
    assert c.get("big") is big and len(c.tabs) == 1 and c.bytes == 10000
    made = []
    for k in range(3):
        c.row(k, lambda: made.append(1) or torch.tensor([k]))
    c.row(2, lambda: made.append(1))
    assert len(made) == 3 and list(c.rows) == [1, 2]
    c.clear()
    assert c.bytes == 0 and not c.tabs and not c.rows
