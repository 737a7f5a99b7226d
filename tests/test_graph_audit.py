"""The region bench.py --graphs captures (GroundingDINO.forward_core and its
backward) builds no tensor from host data: inside a HIP-graph capture such
a copy becomes a memcpy node whose host staging buffer dies with the
capture (tools/graph_h2d_audit.py).  CPU run, HIP-only
ops routed to their oracles; the oracle's own scalar reads are not the
product's and are ignored."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_forward_core_builds_no_tensor_from_host_data(monkeypatch):
    import graph_h2d_audit as audit
    hits = {}
    monkeypatch.setattr(sys, "argv", ["graph_h2d_audit.py"])  # 256 x 320: >= 900 proposals
    orig = audit.Audit.__init__

    def init(self):
        orig(self)
        hits["audit"] = self
    monkeypatch.setattr(audit.Audit, "__init__", init)
    audit.main()
    bad = {k: n for k, n in hits["audit"].hits.items() if k[0] != "_local_scalar_dense"}
    assert not bad, bad


def test_whole_step_body_builds_no_tensor_from_host_data(monkeypatch):
    """The region gdino_amd.stepgraph captures (forward, loss_prepared with
    device matching, weighted loss, backward, clipping): no host-data tensor
    and no device move (the oracle MSDA's own scalar reads aside)."""
    import graph_h2d_audit as audit
    hits = {}
    monkeypatch.setattr(sys, "argv", ["graph_h2d_audit.py", "--whole-step"])
    orig = audit.Audit.__init__

    def init(self):
        orig(self)
        hits["audit"] = self
    monkeypatch.setattr(audit.Audit, "__init__", init)
    audit.main()
    bad = {k: n for k, n in hits["audit"].hits.items() if k[0] != "_local_scalar_dense"}
    assert not bad, bad
