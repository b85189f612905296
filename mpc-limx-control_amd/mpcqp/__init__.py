"""mpcqp -- MI355X-native batched MPC-QP engine (host side).

The compute lives in libmpcqp.so (HIP kernels for gfx950 behind include/mpcqp.h); this
package is the host mirror of the reference's interface for the hot path
(Fleming-Sung/mpc-limX-control: QPSolver, mpcQP, MPCParam) plus the batched engine.
"""
from ._lib import (A_COLMAJOR, A_ROWMAJOR, CONS_BOX, CONS_FRICTION, EXPORTS, LIB_PATH,
                   MODEL_LITERAL, MODEL_SRBM, MPCQP_INFTY, STATUS, MpcqpError, lib)
from .hostmem import page_aligned, page_aligned_empty
from .model import model_params, static_foot_offsets
from .workload import (DEFAULT_SEED, gait_contact_mask, gait_inputs, make_batch,
                       make_gait_states, mpc_test_inputs, qp_harness_inputs)

__all__ = [
    "A_COLMAJOR", "A_ROWMAJOR", "CONS_BOX", "CONS_FRICTION", "EXPORTS", "LIB_PATH",
    "MODEL_LITERAL", "MODEL_SRBM", "MPCQP_INFTY", "STATUS", "MpcqpError", "lib",
    "model_params", "static_foot_offsets", "DEFAULT_SEED", "gait_contact_mask", "make_batch",
    "qp_harness_inputs", "mpc_test_inputs", "gait_inputs", "make_gait_states", "page_aligned",
    "page_aligned_empty",
]
