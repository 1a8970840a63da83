"""CPU oracle for the plainCV transformer training hot path.

TEST INFRASTRUCTURE ONLY.  Nothing under ``oracle/`` is shipped or measured:
only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import it, and there only as the checker.  The product path
(``plaincv_amd``) never routes through this package and fails loudly when the
HIP library is missing.

What it is: a line-by-line PyTorch-CPU restatement (fp32, or fp64 for
finite-difference checks; an optional bf16 "placement" mode that rounds at the
same points as the reference LM's ``dtype: bfloat16``) of the reference's
JAX/Flax/Optax hot path:

* ``oracle.vit``     <- models/vit_small.py:6-127 (+ flax LayerNorm/SelfAttention/Dropout/gelu semantics)
* ``oracle.lm``      <- models/LM/transformer.py:32-407, models/LM/embedding.py:8-66
* ``oracle.engine``  <- engine/flax_engine.py:13-134, train_lm.py:134-353
* ``oracle.optim``   <- optim/factory.py:193-205,441-484,632-673; optim/muon.py:120-129;
                        optim/matrix_routing.py:8-40; optim/soap.py:15-368; optim/shampoo.py:81-296
                        (+ optax 0.2.6 adamw / contrib.muon semantics)
* ``oracle.rng``     the counter-based dropout hash shared with the HIP kernels
                     (the reference's threefry stream cannot be reproduced without JAX).

PARITY UNPINNED: the reference publishes no golden vectors or tests for this
path and JAX/Flax/Optax are not installed here, so the
restatement cannot be checked against reference outputs.  It is anchored
instead by the closed-form known-answer tests in tests/test_oracle_*.py
 and by fixtures generated from it
(tests/golden/make_golden.py).
"""
