"""Mirror of ``pldepth.data.dao``: on-disk dataset access for training."""
