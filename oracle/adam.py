"""Adam(amsgrad=True) update — TEST INFRASTRUCTURE (see oracle/__init__).

Restates keras.optimizers.Adam(learning_rate, amsgrad=True) (pldepth/PLDepth.py:133) as TF
applies it per variable (ResourceApplyAdamWithAmsgrad functor; Keras defaults beta_1=0.9,
beta_2=0.999, epsilon=1e-7; local_step = iterations + 1; all in float32):
    alpha = lr * sqrt(1 - b2^t) / (1 - b1^t)
    m += (g - m) * (1 - b1);  v += (g*g - v) * (1 - b2);  vhat = max(vhat, v)
    p -= m * alpha / (sqrt(vhat) + eps)
"""
import numpy as np


def adam_amsgrad_step(p, g, m, v, vhat, lr, step, beta1=0.9, beta2=0.999, eps=1e-7):
    f = np.float32
    p, g, m, v, vhat = (np.asarray(a, np.float32).copy() for a in (p, g, m, v, vhat))
    b1p = f(np.power(f(beta1), f(step)))
    b2p = f(np.power(f(beta2), f(step)))
    alpha = f(f(lr) * np.sqrt(f(1) - b2p) / (f(1) - b1p))
    m += (g - m) * (f(1) - f(beta1))  # TF: T(1) - beta1 with float32 beta1
    v += (g * g - v) * (f(1) - f(beta2))
    vhat = np.maximum(vhat, v)
    p -= (m * alpha) / (np.sqrt(vhat) + f(eps))
    return p, m, v, vhat
