"""DnCNN training driver (mirror of /root/reference/main_train_dncnn.py:46-250; BASELINE config 1).

    python -m kair_amd.main_train_dncnn -opt options/train_dncnn.json

Same loop as the reference: parse -> find_last_checkpoint -> seeds -> DatasetDnCNN + DataLoader ->
define_Model (ModelPlain) -> merge_bnorm_test when resuming past merge_bn_startpoint -> init_train
-> per step: update_learning_rate (before the step, :163), feed_data, optimize_parameters,
merge_bnorm_train at merge_bn_startpoint (:179-182), log / save / test (PSNR on uint8, border 0).
gpu_ids null runs it on the host (config 1's "plumbing, no GPU"); gpu_ids [0] on the MI355X.
Additions: train.max_iter ends the run (the reference loops until killed); train.manual_seed.
"""
import argparse
import logging
import math
import os
import random
import sys

import numpy as np
import torch
from torch.utils.data import DataLoader

from .data.select_dataset import define_Dataset
from .models.select_model import define_Model
from .utils import utils_image as util
from .utils import utils_option as option


def main(json_path="options/train_dncnn.json", overrides=None, log_stream=None):
    opt = option.parse(json_path, is_train=True)
    if overrides:
        overrides(opt)
    for key, path in opt["path"].items():
        if "pretrained" not in key and isinstance(path, str):
            os.makedirs(path, exist_ok=True)
    init_iter, init_path_G = option.find_last_checkpoint(opt["path"]["models"], net_type="G")
    opt["path"]["pretrained_netG"] = init_path_G
    current_step = init_iter
    border = 0
    option.save(opt)
    opt = option.dict_to_nonedict(opt)

    logger = logging.getLogger("kair_amd.train_dncnn")
    if not logger.handlers:
        logger.setLevel(logging.INFO)
        logger.addHandler(logging.StreamHandler(log_stream or sys.stdout))

    seed = opt["train"]["manual_seed"]
    if seed is None:
        seed = random.randint(1, 10000)
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)

    train_loader = test_loader = None
    for phase, ds in opt["datasets"].items():
        dset = define_Dataset(ds)
        if phase == "train":
            logger.info("Number of train images: {:,d}, iters: {:,d}".format(
                len(dset), int(math.ceil(len(dset) / ds["dataloader_batch_size"]))))
            train_loader = DataLoader(dset, batch_size=ds["dataloader_batch_size"], shuffle=ds["dataloader_shuffle"],
                                      num_workers=ds["dataloader_num_workers"] or 0, drop_last=True,
                                      pin_memory=torch.cuda.is_available())
        elif phase == "test":
            test_loader = DataLoader(dset, batch_size=1, shuffle=False, num_workers=0, drop_last=False)

    model = define_Model(opt)
    if opt["merge_bn"] and current_step > opt["merge_bn_startpoint"]:
        logger.info("^_^ -----merging bnorm----- ^_^")
        model.merge_bnorm_test()
    model.init_train()

    max_iter = opt["train"]["max_iter"]
    history = {"loss": [], "psnr": []}
    done = False
    for epoch in range(1000000):
        for train_data in train_loader:
            current_step += 1
            model.update_learning_rate(current_step)
            model.feed_data(train_data)
            model.optimize_parameters(current_step)
            history["loss"].append(model.current_log()["G_loss"])
            if opt["merge_bn"] and opt["merge_bn_startpoint"] == current_step:
                logger.info("^_^ -----merging bnorm----- ^_^")
                model.merge_bnorm_train()
            if current_step % opt["train"]["checkpoint_print"] == 0:
                msg = "<epoch:{:3d}, iter:{:8,d}, lr:{:.3e}> ".format(epoch, current_step, model.current_learning_rate())
                msg += " ".join("{:s}: {:.3e}".format(k, v) for k, v in model.current_log().items())
                logger.info(msg)
            if current_step % opt["train"]["checkpoint_save"] == 0:
                model.save(current_step)
            if test_loader is not None and current_step % opt["train"]["checkpoint_test"] == 0:
                avg = 0.0
                for idx, test_data in enumerate(test_loader, 1):
                    model.feed_data(test_data)
                    model.test()
                    vis = model.current_visuals()
                    avg += util.calculate_psnr(util.tensor2uint(vis["E"]), util.tensor2uint(vis["H"]), border=border)
                avg /= idx
                history["psnr"].append((current_step, avg))
                logger.info("<epoch:{:3d}, iter:{:8,d}, Average PSNR : {:<.2f}dB".format(epoch, current_step, avg))
            if max_iter is not None and current_step >= max_iter:
                done = True
                break
        if done:
            break
    model.save("latest")
    return model, history


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-opt", type=str, default="options/train_dncnn.json")
    main(ap.parse_args().opt)
