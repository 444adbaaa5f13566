"""Optimizer configuration (mirrors ``keras.optimizers.Adam(learning_rate, amsgrad=True)``,
pldepth/PLDepth.py:133). The update itself is the fused HIP kernel pld_adam_amsgrad_dev; this
object carries the hyper-parameters and the current learning rate (``lr``), which callbacks such
as ``SGDRScheduler`` set per batch (training_utils.py:80-88), exactly like K.set_value(...lr).
"""


class Adam(object):
    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-7, amsgrad=False,
                 name="Adam"):
        if not amsgrad:
            raise NotImplementedError("PLDepth trains with Adam(amsgrad=True) only")
        self.lr = float(learning_rate)
        self.beta_1, self.beta_2, self.epsilon = float(beta_1), float(beta_2), float(epsilon)
        self.amsgrad = True
        self.iterations = 0
        self.name = name

    @property
    def learning_rate(self):
        return self.lr

    @learning_rate.setter
    def learning_rate(self, v):
        self.lr = float(v)

    def get_config(self):
        return {"learning_rate": self.lr, "beta_1": self.beta_1, "beta_2": self.beta_2,
                "epsilon": self.epsilon, "amsgrad": True}
