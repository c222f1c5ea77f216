"""Canonical digest of a rendered ACL rule list (every field of every rule
message, in order), used to pin the benchmark tables against process history."""
import dataclasses
import hashlib


def rule_list_digest(rules) -> str:
    m = hashlib.sha256()
    for r in rules:
        m.update(repr(dataclasses.astuple(r)).encode())
        m.update(b"\n")
    return m.hexdigest()
