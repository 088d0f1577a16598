"""TEST INFRASTRUCTURE ONLY — CPU oracle for the conditional-RealNVP hot path.

Nothing in the product package (`arl_conditional_normalizing_flows_amd`) imports
this package. Only `tests/`, `__graft_entry__.smoke()` and the `cpu_baseline`
leg of `bench.py` may use it, and only as the checker / the timed CPU baseline.

Parity status: **parity unpinned** (against the reference itself).
The reference (USArmyResearchLab/ARL_Conditional_Normalizing_Flows) is pure
TensorFlow/Keras/TFP Python; TF is not installed in this image (an ordinary
`ModuleNotFoundError`, not a permission denial — SURVEY.md §8(c)) and the
reference ships no tests, fixtures or golden vectors. This oracle is a
from-scratch restatement of the reference source (every function cites the
file:line it follows) plus the documented Keras/TF semantics the reference
relies on (LeakyReLU alpha=0.3, LayerNormalization eps=1e-3, Conv2D 'same'
padding / HWIO kernels, `space_to_depth` channel order, MVNDiag log-prob).
It is pinned only by analytic known-answer invariants (tests/test_oracle.py):
round trip, brute-force Jacobian log-det, zero-weight identity, permutation
bijectivity.

Modules
-------
cflow_np         numpy float64/float32 restatement of `cFlow` (the checker)
cflow_torch_cpu  torch-CPU fp32 op-for-op restatement (the timed CPU baseline)
toy_np           numpy restatement of the dense toy `cINN_affine` (config 1)
"""
