def check_space(space, space_type, check_box_space_fn):  # placeholder; ap_gym.make swaps it out temporarily
    return None
