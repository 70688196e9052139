"""kair_amd — MI355X-native (gfx950) training/inference path for KAIR's image-restoration networks.

Drop-in surface (mirrors Owen1B/KAIR): kair_amd.models.select_network.define_G,
kair_amd.models.select_model.define_Model, ModelPlain / ModelPlain4, kair_amd.utils.utils_option.
Compute: libkair_hip.so (kair_amd/csrc, C ABI in include/kair_hip.h), no CPU fallback.
"""
__version__ = "0.1.0"
