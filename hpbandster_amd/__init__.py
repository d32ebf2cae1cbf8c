"""hpbandster_amd: MI355X-native engine for HpBandSter's data-parallel hot path.

* ``kde``       -- device-resident BOHB KDE models: refit, fp32 matrix-core scoring, exact argmin
* ``promote``   -- batched successive-halving promotion (segmented top-k)
* ``config_generators`` -- BOHB / KDEEI / RandomSampling drop-ins (get_config / new_result)
* ``HB_iteration`` / ``HB_master`` / ``HB_result`` -- the Hyperband API
* ``distributed`` -- candidate sharding over GPUs with one RCCL exchange of the local winners

The compute path is libhbx.so (HIP, gfx950); there is no CPU fallback.
"""
__version__ = "0.1.0"
