"""Expected results of the build's own codecs, restated with the oracle (test helper)."""
import numpy as np
import torch

MICRO_Q8_CAP = 3 * 4096  # bucket cap for the int8-wire tests: 3+ buckets on the micro tree


def expected_q8(n, steps=2, cap=MICRO_Q8_CAP):
    """The int8-wire outer step restated with the oracle (tests/oracle_kernels.py layout)."""
    from diloco_amd import synth
    from diloco_amd.trees import get_tree
    from oracle import oracle
    from oracle_kernels import OracleKernels

    spec = get_tree("micro")
    numels = spec.numels()
    tree = OracleKernels().tree(numels, torch.device("cpu"), cap)
    counts = [c1 - c0 for c0, c1 in tree.bucket_chunks]
    theta = synth.outer_tree(numels, spec.init_spec())
    buf = [np.empty_like(t) for t in theta]
    out = {}
    for s in range(1, steps + 1):
        deltas = [[oracle.delta(t, i) for t, i in zip(theta, synth.inner_tree(theta, s, r))]
                  for r in range(n)]
        g = oracle.q8_average(deltas, numels, counts)
        for t in range(len(theta)):
            oracle.sgd(theta[t], buf[t], g[t], 0.7, 0.9, True, s == 1)
        out[f"theta_s{s}"] = np.concatenate(theta)
    return out


def expected_rank_order(n, steps=2, wire="f32"):
    """The outer step with the replicas' deltas summed in rank order in fp32 (a bf16 wire
    rounds each delta first and never the sum): oracle.OuterState, micro tree, n replicas --
    what exchange="a2a" and the direct exchange compute at every n."""
    from diloco_amd import synth
    from diloco_amd.trees import get_tree
    from oracle import oracle

    spec = get_tree("micro")
    theta0 = synth.outer_tree(spec.numels(), spec.init_spec())
    st = oracle.OuterState(theta0)
    out = {}
    for s in range(1, steps + 1):
        inners = [synth.inner_tree(st.theta, s, r) for r in range(n)]
        st.step(inners, wire)
        out[f"theta_s{s}"] = np.concatenate(st.theta)
        out[f"buf_s{s}"] = np.concatenate(st.buf)
    return out
