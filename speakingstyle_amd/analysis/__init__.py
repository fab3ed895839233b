"""Research tooling that the reference keeps in notebooks: variance (pitch / energy /
duration) distribution analysis of ground truth vs model predictions
(``notebooks/variance_control_distbn.ipynb``) and a one-batch forward / style-encoder
inspection on the training data (``notebooks/ref_encoder.ipynb``)."""
