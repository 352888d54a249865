from .nccl_p2p import (add_delay, get_unique_nccl_id, init_nccl_comm, left_right_halo_exchange,
                       left_right_halo_exchange_inplace)
