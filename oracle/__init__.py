"""TEST INFRASTRUCTURE ONLY: the C restatement of the reference path (parity oracle)."""
