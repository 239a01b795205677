"""MI355X-native vehicle-pass imaging hot path of NohPei/das_diff_veh (VSG -> class stack -> f-v).

Submodules mirror the reference layout: ``apis.virtual_shot_gather``, ``apis.dispersion_classes``,
``apis.data_classes``, ``apis.imaging_classes`` and ``modules.utils``.  Compute runs in hand-written
HIP kernels behind the C-ABI library ``libdvh.so`` (see ``include/dvh.h``); this package never
falls back to a CPU path.
"""
__version__ = "0.1.0"
