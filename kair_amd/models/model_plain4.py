"""ModelPlain4 — four-input trainer for USRNet (mirror of /root/reference/models/model_plain4.py:11-23).

The reference's feed_data uses np.int (removed in numpy 1.24, SURVEY.md §0 gotcha 4); the scale
factor is read with int() here.  optimize_parameters runs the fused trainer (USRNet step program +
L1 + fused Adam/EMA, one HIP graph per step) with (k, sf, sigma) as the step's extra inputs.
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

    def _step_cond(self):
        """USRNet's extra forward inputs (model_plain4.py:22-23) for the fused, graph-captured step."""
        return (self.k, self.sf, self.sigma)

    def netG_forward(self):
        self.E = self.netG(self.L, self.k, self.sf, self.sigma)
