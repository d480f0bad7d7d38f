"""ace_amd -- MI355X-native 2ACE ADMM channel recovery (HIP kernels behind a C-ABI).

Importing this package loads ``libace.so``; it raises if the HIP library has
not been built (there is no CPU fallback on the product path).
"""
from ._lib import LIB, AceError, AdmmCfg, default_cfg  # noqa: F401
from ._lib import (ACE_VARIANT_A2ONLY, ACE_VARIANT_NUCLEAR, ACE_ST_CONVERGED, ACE_ST_NO_OPT,  # noqa: F401
                   ACE_ST_EIG_NOCONV, ACE_ST_ROLLBACK, PipelineCfg, pipeline_cfg)
from .solver import (InferADMM, infer_admm_batch, infer_admm_host, synth_problem, BatchResult,  # noqa: F401
                     nuclear_prox_batch)
from ._lib import path_counts  # noqa: F401
from .pipeline import (inferLowRankV4_multi, inferLowRankV4, inferLowRank_Nuclear,  # noqa: F401
                       infer_low_rank_pipeline_host, infer_low_rank_pipeline_batch, draw_partitions,
                       PipelineResult, SpectralInitialize)
from .phaselift import MyPhaseLift, phaselift_host, phaselift_batch, PhaseLiftResult, prox_eig_host  # noqa: F401
from .beamformer import (svd_beamformer, svd_beamformer_compensation, codebook_beams,  # noqa: F401
                         svd_beamformer_host, svd_beamformer_batch, BeamResult)
from . import synth, engine  # noqa: F401

__version__ = LIB.ace_version().decode()
