"""Pin the oracle to the reference's own known-answer tests (CPU)."""
import pytest

import kat_runner as K

CASES = [(f, c) for f in ("kat_vclock.json", "kat_counters.json", "kat_orswot.json", "kat_mvreg.json")
         for c in K.load_cases(f)]


@pytest.mark.parametrize("fname,case", CASES, ids=[c["name"] for _, c in CASES])
def test_kat_oracle(fname, case):
    K.run_case(case)
