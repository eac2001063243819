"""MI355X-native DiLoCo outer-step sync for mikasenghaas/diloco-swarm.

Drop-in modules mirroring the reference's call surface:
  diloco_amd.comm        TrainingComm / InferenceComm      (src/comm.py)
  diloco_amd.serializer  Serializer / Metadata             (src/serializer.py)
  diloco_amd.utils       get_outer_model, compute_pseudo_gradient, sync_inner_model,
                         get_optimizer                     (src/utils.py:59-65, 203-226)
  diloco_amd.world       World                             (src/world.py)
Engines: diloco_amd.outer.OuterSync (device-resident outer step), diloco_amd.gradsync.GradSync
(DP average of device gradients), diloco_amd.mirror.HostOuterMirror (device mirror of the
host outer model). Native code: libdiloco_hip.so (include/diloco_hip.h) via diloco_amd._lib.
"""
__version__ = "0.1.0"
