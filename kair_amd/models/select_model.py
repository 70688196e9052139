"""define_Model (mirror of /root/reference/models/select_model.py:9-33).

'plain' (one input) and 'plain4' (USRNet: L, k, sf, sigma) are on the MI355X path; the GAN / video
trainers ('gan', 'vrt', 'plain2') are out of scope and raise NotImplementedError.
"""


def define_Model(opt):
    model = opt["model"]
    if model == "plain":
        from .model_plain import ModelPlain as M
    elif model == "plain4":
        from .model_plain4 import ModelPlain4 as M
    else:
        raise NotImplementedError("Model [{:s}] is not on the kair_amd MI355X path.".format(model))
    m = M(opt)
    print("Training model [{:s}] is created.".format(m.__class__.__name__))
    return m
