"""Mirror of ``pldepth.active_learning``: the test-pass metrics the training script reports."""
