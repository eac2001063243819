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
        out[f"buf_s{s}"] = np.concatenate(buf)
        out[f"avg_s{s}"] = np.concatenate(g)
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
        _, avg = st.step(inners, wire)
        out[f"avg_s{s}"] = np.concatenate(avg)
        out[f"theta_s{s}"] = np.concatenate(st.theta)
        out[f"buf_s{s}"] = np.concatenate(st.buf)
    return out


def expected_bf16_allreduce(n, steps=2):
    """The outer step with a bf16 wire summed by the transport in bf16 (RCCL's / gloo's bf16
    SUM: each replica's delta rounded to bf16, every partial sum rounded to bf16, in rank order)
    and averaged in fp32 -- what the fused device outer model with wire="bf16" computes; the
    order of the partial sums does not matter at n = 2. Micro tree; returns θ, the momentum
    and the decoded average g (what .grad shows) per step."""
    from diloco_amd import synth
    from diloco_amd.trees import get_tree
    from oracle import oracle

    spec = get_tree("micro")
    theta = [t.copy() for t in synth.outer_tree(spec.numels(), spec.init_spec())]
    buf = [np.empty_like(t) for t in theta]
    out = {}
    for s in range(1, steps + 1):
        inners = [synth.inner_tree(theta, s, r) for r in range(n)]
        avg = []
        for t in range(len(theta)):
            d = [oracle.bf16_round(oracle.delta(theta[t], inners[r][t])) for r in range(n)]
            acc = d[0]
            for dr in d[1:]:
                acc = oracle.bf16_round((acc + dr).astype(np.float32))
            g = (acc / np.float32(n)).astype(np.float32)
            oracle.sgd(theta[t], buf[t], g, 0.7, 0.9, True, s == 1)
            avg.append(g)
        out[f"theta_s{s}"] = np.concatenate(theta)
        out[f"buf_s{s}"] = np.concatenate(buf)
        out[f"avg_s{s}"] = np.concatenate(avg)
    return out
