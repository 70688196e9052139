"""ModelPlain4 — four-input trainer for USRNet (mirror of /root/reference/models/model_plain4.py:11-23).

The reference's feed_data uses np.int (removed in numpy 1.24, SURVEY.md §0 gotcha 4); the scale
factor is read with int() here.
"""
from .model_plain import ModelPlain


class ModelPlain4(ModelPlain):
    def feed_data(self, data, need_H=True):
        self.L = data["L"].to(self.device)
        self.k = data["k"].to(self.device)
        self.sf = int(data["sf"][0, ...].squeeze().cpu().item())
        self.sigma = data["sigma"].to(self.device)
        if need_H:
            self.H = data["H"].to(self.device)

    def _fused_ok(self):
        return False   # USRNet trains through the autograd node (its step is not graph-captured yet)

    def netG_forward(self):
        self.E = self.netG(self.L, self.k, self.sf, self.sigma)
