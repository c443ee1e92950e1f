"""InferenceWrapper — drop-in for reference models/inference_wrapper.py:4-25.

Same constructor and forward contract: a CHW image -> (binary one-hot mask [2,H,W], sigmoid
probabilities [2,H,W]) from the model's first logit map, bilinearly resized (align_corners=False) to
the image size.  The resize is the device bilinear kernel (ssseg_bilinear_fwd) and the sigmoid +
argmax/one-hot head is one kernel (ssseg_prob_onehot); there is no CPU path.
"""
import torch
import torch.nn as nn

from ssseg import ops


class InferenceWrapper(nn.Module):
    def __init__(self, model):
        super(InferenceWrapper, self).__init__()
        self.model = model

    def forward(self, image):
        # image: 3d image of shape CxHxW (inference_wrapper.py:9-10)
        image = torch.unsqueeze(image, 0)
        features, logit_resolutions = self.model(image)
        high_resolution_logits = logit_resolutions[0]
        high_resolution_logits = ops.interpolate_bilinear(high_resolution_logits.float(),
                                                          [image.size(2), image.size(3)], align_corners=False)
        probabilities, binary_mask_nchw = ops.prob_onehot(high_resolution_logits)
        return binary_mask_nchw[0], probabilities[0]
