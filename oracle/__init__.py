"""CPU oracle for the semi-supervised segmentation training hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product (semi-supervised_semantic_segmentation_amd/)
imports this package.  Only tests/, __graft_entry__.smoke() and bench.py's `cpu_baseline` leg may
use it, and only as the checker / the CPU baseline — never as a fallback for the HIP path.

It restates the reference's algorithm (Luonic/semi-supervised_semantic_segmentation, mounted at
/root/reference in the build container) function by function; every function cites the reference
file:line it follows.  Byte/float-order sensitive pieces (CowMix filter, Lovász, consistency, EMA,
BCE, bilinear interpolation) are numpy; the network graphs and the training step are torch-CPU
(fp32), which is the reference's own CPU arithmetic.

Pinning: the restatement is checked against golden vectors generated from the reference itself
(tests/golden/gen_golden.py, fixtures G1-G7) by tests/test_oracle_golden.py.  Pieces that the
reference cannot pin (the ResNet-50 encoder, which the reference lacks — SURVEY §0.4) are marked
"parity unpinned" where they are defined.
"""
