"""Drop-in ``Decoder`` (model/decoder.py:15).

Same module structure (``layers`` ModuleList + ``lout``) so state_dict keys
``layers.{i}.weight/bias`` and ``lout.weight/bias`` load unchanged, and the same
``sdf`` / ``occupancy`` / ``sem_label_prob`` / ``regress_color`` heads.  The
fused tracker/mesher/mapper kernels read the geo decoder's weights directly
(pin_slam_amd.query.mlp_view); ``sdf`` itself is the plain module forward used
by callers that go through ``NeuralPoints.query_feature``.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


class Decoder(nn.Module):
    def __init__(self, config, hidden_dim, hidden_level, out_dim, is_time_conditioned=False):
        super().__init__()
        self.out_dim = out_dim
        bias_on = config.mlp_bias_on
        self.use_leaky_relu = False
        self.num_bands = config.pos_encoding_band
        self.dimensionality = config.pos_input_dim
        if config.use_gaussian_pe:
            position_dim = config.pos_input_dim + 2 * config.pos_encoding_band
        else:
            position_dim = config.pos_input_dim * (2 * config.pos_encoding_band + 1)
        in_dim = config.feature_dim + position_dim + (1 if is_time_conditioned else 0)
        self.layers = nn.ModuleList(
            [nn.Linear(in_dim if i == 0 else hidden_dim, hidden_dim, bias_on) for i in range(hidden_level)])
        self.lout = nn.Linear(hidden_dim, out_dim, bias_on)
        if config.main_loss_type == "bce":
            self.sdf_scale = config.logistic_gaussian_ratio * config.sigma_sigmoid_m
        else:
            self.sdf_scale = 1.0
        self.to(config.device)

    def forward(self, feature):
        return self.sdf(feature)

    def _trunk(self, x):
        act = F.leaky_relu if self.use_leaky_relu else F.relu
        for layer in self.layers:
            x = act(layer(x))
        return x

    def sdf(self, features):
        """model/decoder.py:66-88 (prediction is the scaled sdf)."""
        out = self.lout(self._trunk(features)).squeeze(1)
        return out * self.sdf_scale

    def time_conditionded_sdf(self, features, ts):
        nn_k = features.shape[1]
        ts_nn_k = ts.repeat(nn_k).view(-1, nn_k, 1)
        out = self.lout(self._trunk(torch.cat((features, ts_nn_k), dim=-1))).squeeze(1)
        return out * self.sdf_scale

    def occupancy(self, features):
        return torch.sigmoid(self.sdf(features) / -self.sdf_scale)

    def sem_label_prob(self, features):
        return F.log_softmax(self.lout(self._trunk(features)), dim=-1)

    def sem_label(self, features):
        return torch.argmax(self.sem_label_prob(features), dim=1)

    def regress_color(self, features):
        return torch.clamp(self.lout(self._trunk(features)), 0.0, 1.0)
