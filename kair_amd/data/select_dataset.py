"""Dataset factory (mirror of /root/reference/data/select_dataset.py:12-100) for the datasets that
feed the kair_amd hot path: 'dncnn' (DatasetDnCNN, config 1) and 'sr' (DatasetSR, configs 2/4/5).
Other dataset types are off the path and raise NotImplementedError naming the type."""


def define_Dataset(dataset_opt):
    t = dataset_opt["dataset_type"].lower()
    if t in ("dncnn", "denoising"):
        from .dataset_dncnn import DatasetDnCNN as D
    elif t in ("sr", "super-resolution"):
        from .dataset_sr import DatasetSR as D
    else:
        raise NotImplementedError(f"Dataset [{t}] is not on the kair_amd path (dncnn, sr).")
    return D(dataset_opt)
