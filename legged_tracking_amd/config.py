"""Config contract of the reference (Cfg / config_go1) and its mapping onto the C ABI.

`Cfg` mirrors go1_gym/envs/base/legged_robot_trajectory_tracking_config.py:6-373
(the attributes the trajectory-tracking step reads); `config_go1` mirrors
go1_gym/envs/go1/go1_crawling.py:8-106.  Both are plain mutable classes so that
scripts/train.py:46-241 can mutate them exactly as it mutates the reference's
params_proto classes.  `vars(Cfg.x)` returns a new dict of public attributes in
definition order (the reading of params_proto 2.10.5's Meta.__dict__ used by
the survey; params_proto itself is absent offline).

`build_abi_config()` turns a mutated Cfg into the go1_config struct, computing
every constant the way torch would (f32 scalars, same operation order).
"""
import math

import numpy as np

from . import abi, layout as L, model as M

_TYPE_DICT = type.__dict__["__dict__"]


class _Meta(type):
    """vars(cls) -> fresh dict of public non-callable class attributes."""

    @property
    def __dict__(cls):
        out = {}
        for k, v in _TYPE_DICT.__get__(cls).items():
            if k.startswith("_") or isinstance(v, (type, staticmethod, classmethod, property)) or callable(v):
                continue
            out[k] = v
        return out


class PrefixProto(metaclass=_Meta):
    def __init_subclass__(cls, **kwargs):
        pass


ParamsProto = PrefixProto


def make_cfg():
    """A fresh Cfg class tree with the reference's defaults (config.py:6-373)."""

    class Cfg(PrefixProto, cli=False):
        class env(PrefixProto, cli=False):
            num_envs = 4096
            num_observations = 235
            num_scalar_observations = 42
            num_privileged_obs = 6
            privileged_future_horizon = 1
            num_actions = 12
            num_observation_history = 15
            env_spacing = 3.
            send_timeouts = True
            episode_length_s = 20
            observe_heights = True
            observe_vel = True
            observe_only_ang_vel = False
            observe_only_lin_vel = False
            observe_yaw = False
            observe_contact_states = False
            observe_command = True
            observe_height_command = True
            observe_gait_commands = False
            observe_timing_parameter = False
            observe_clock_inputs = False
            observe_two_prev_actions = False
            observe_imu = False
            record_video = True
            recording_width_px = 360
            recording_height_px = 240
            recording_mode = "COLOR"
            num_recording_envs = 1
            debug_viz = False
            all_agents_share = False
            look_from_back = False
            priv_observe_friction = True
            priv_observe_friction_indep = True
            priv_observe_ground_friction = False
            priv_observe_ground_friction_per_foot = False
            priv_observe_restitution = True
            priv_observe_base_mass = True
            priv_observe_com_displacement = True
            priv_observe_motor_strength = False
            priv_observe_motor_offset = False
            priv_observe_joint_friction = True
            priv_observe_Kp_factor = True
            priv_observe_Kd_factor = True
            priv_observe_contact_forces = False
            priv_observe_contact_states = False
            priv_observe_body_velocity = False
            priv_observe_foot_height = False
            priv_observe_body_height = False
            priv_observe_gravity = False
            priv_observe_terrain_type = False
            priv_observe_clock_inputs = False
            priv_observe_doubletime_clock_inputs = False
            priv_observe_halftime_clock_inputs = False
            priv_observe_desired_contact_states = False
            priv_observe_dummy_variable = False
            terminate_end_of_trajectory = False
            use_terminal_body_rotation = False
            rotate_camera = False
            camera_zero = True
            command_xy_only = True
            viewer_look_at_robot = False

        class terrain(PrefixProto, cli=False):
            mesh_type = 'trimesh'
            terrain_type = 'random_pyramid'
            valid_tunnel_only = False
            ceiling_height = 0.5
            start_loc = 0.4
            x_init_range = 0.
            y_init_range = 0.
            x_init_offset = 0.
            y_init_offset = 0.
            yaw_init_range = 0.
            static_friction = 1.0
            dynamic_friction = 1.0
            restitution = 0.
            terrain_ratio_x = 0.5
            terrain_ratio_y = 0.5
            terrain_length = 8.0
            terrain_width = 3.6
            terrain_border_ratio_x = 0.9
            terrain_border_ratio_y = 0.5
            num_rows = 1
            num_cols = 1
            horizontal_scale = 0.05
            vertical_scale = 0.005
            measured_points_x = np.linspace(-1, 1, 21)
            measured_points_y = np.linspace(-0.5, 0.5, 11)
            measure_front_half = True
            terminate_end_of_trajectory = False

        class commands(PrefixProto, cli=False):
            switch_upon_reach = True
            switch_interval = 0.5
            traj_function = "fixed_target"
            traj_length = 1
            num_interpolation = 1
            base_x = 5.0
            base_y = 0.0
            base_z = 0.34
            base_roll = 0.0
            base_pitch = 0.0
            base_yaw = 0.0
            x_range = 0.4
            y_range = 0.5
            z_range = 0.1
            roll_range = 30 * np.pi / 180
            pitch_range = 30 * np.pi / 180
            yaw_range = 180 * np.pi / 180
            x_mean = 3.6
            y_mean = 3.6
            y_eang = 0.4
            global_reference = False
            switch_dist = 0.05
            switch_yaw = 0.5
            sampling_based_planning = False
            plan_interval = 10

        class curriculum_thresholds(PrefixProto, cli=False):
            cl_fix_target = False
            cl_start_target_dist = 0.5
            cl_goal_target_dist = 3.6
            cl_switch_delta = 0.5
            cl_switch_threshold = 1.0

        class init_state(PrefixProto, cli=False):
            pos = [0.0, 0.0, 1.]
            rot = [0.0, 0.0, 0.0, 1.0]
            lin_vel = [0.0, 0.0, 0.0]
            ang_vel = [0.0, 0.0, 0.0]
            default_joint_angles = {"joint_a": 0., "joint_b": 0.}

        class control(PrefixProto, cli=False):
            control_type = 'actuator_net'
            stiffness = {'joint_a': 10.0, 'joint_b': 15.}
            damping = {'joint_a': 1.0, 'joint_b': 1.5}
            action_scale = 0.5
            hip_scale_reduction = 1.0
            decimation = 4

        class asset(PrefixProto, cli=False):
            file = ""
            foot_name = "None"
            penalize_contacts_on = []
            terminate_after_contacts_on = []
            disable_gravity = False
            collapse_fixed_joints = True
            fix_base_link = False
            default_dof_drive_mode = 3
            self_collisions = 0
            replace_cylinder_with_capsule = True
            flip_visual_attachments = True
            density = 0.001
            angular_damping = 0.
            linear_damping = 0.
            max_angular_velocity = 1000.
            max_linear_velocity = 1000.
            armature = 0.
            thickness = 0.01

        class domain_rand(PrefixProto, cli=False):
            rand_interval_s = 10
            randomize_motor_strength = False
            randomize_motor_offset = True
            motor_offset_range = [-0.02, 0.02]
            randomize_rigids_after_start = True
            randomize_friction = True
            friction_range = [0.5, 1.25]
            randomize_restitution = False
            restitution_range = [0, 1.0]
            randomize_base_mass = False
            added_mass_range = [-1., 1.]
            randomize_com_displacement = False
            com_displacement_range = [-0.15, 0.15]
            motor_strength_range = [0.9, 1.1]
            randomize_Kp_factor = False
            Kp_factor_range = [0.8, 1.3]
            randomize_Kd_factor = False
            Kd_factor_range = [0.5, 1.5]
            gravity_rand_interval_s = 7
            gravity_impulse_duration = 1.0
            randomize_gravity = False
            gravity_range = [-1.0, 1.0]
            push_robots = True
            push_interval_s = 15
            max_push_vel_xy = 1.
            randomize_lag_timesteps = True
            lag_timesteps = 6

        class rewards(PrefixProto, cli=False):
            only_positive_rewards = True
            only_positive_rewards_ji22_style = False
            sigma_rew_neg = 5
            reward_container_name = "RewardsCrawling"
            target_lin_vel = 0.5
            lin_reaching_criterion = 0.1
            tracking_sigma_lin = 0.10
            target_ang_vel = np.pi / 2.0
            ang_reaching_criterion = np.pi / 20.
            tracking_sigma_ang = 0.5
            use_terminal_body_height = True
            terminal_body_height = 0.1

        class reward_scales(ParamsProto, cli=False):
            torques = -0.00001
            dof_acc = -2.5e-7
            collision = -1.
            action_rate = -0.01
            reaching_linear_vel = 0.0
            reaching_z = 0.0
            reaching_yaw = 0.0

        class normalization(PrefixProto, cli=False):
            clip_observations = 100.
            clip_actions = 100.
            friction_range = [0.05, 4.5]
            ground_friction_range = [0.05, 4.5]
            restitution_range = [0, 1.0]
            added_mass_range = [-1., 3.]
            com_displacement_range = [-0.1, 0.1]
            motor_strength_range = [0.9, 1.1]
            motor_offset_range = [-0.05, 0.05]
            Kp_factor_range = [0.8, 1.3]
            Kd_factor_range = [0.5, 1.5]
            joint_friction_range = [0.0, 0.7]
            contact_force_range = [0.0, 50.0]
            contact_state_range = [0.0, 1.0]
            body_velocity_range = [-6.0, 6.0]
            foot_height_range = [0.0, 0.15]
            body_height_range = [0.0, 0.60]
            gravity_range = [-1.0, 1.0]
            motion = [-0.01, 0.01]

        class obs_scales(PrefixProto, cli=False):
            lin_vel = 2.0
            ang_vel = 0.25
            dof_pos = 1.0
            dof_vel = 0.05
            imu = 0.1
            height_measurements = 0.1
            friction_measurements = 1.0

        class noise(PrefixProto, cli=False):
            add_noise = True
            noise_level = 1.0

        class noise_scales(PrefixProto, cli=False):
            dof_pos = 0.01
            dof_vel = 1.5
            lin_vel = 0.1
            ang_vel = 0.2
            imu = 0.1
            gravity = 0.05
            contact_states = 0.05
            height_measurements = 0.1
            friction_measurements = 0.0

        class viewer(PrefixProto, cli=False):
            ref_env = 0
            pos = [10, 0, 6]
            lookat = [11., 5, 3.]

        class sim(PrefixProto, cli=False):
            dt = 0.005
            substeps = 1
            gravity = [0., 0., -9.81]
            up_axis = 1
            use_gpu_pipeline = True

            class physx(PrefixProto, cli=False):
                num_threads = 10
                solver_type = 1
                num_position_iterations = 4
                num_velocity_iterations = 0
                contact_offset = 0.01
                rest_offset = 0.0
                bounce_threshold_velocity = 0.5
                max_depenetration_velocity = 1.0
                max_gpu_contact_pairs = 2 ** 23
                default_buffer_size_multiplier = 5
                contact_collection = 2

    return Cfg


Cfg = make_cfg()


def config_go1(Cnfg):
    """go1_gym/envs/go1/go1_crawling.py:8-106 (values only)."""
    _ = Cnfg.init_state
    _.pos = [0.0, 0.0, 0.34]
    _.default_joint_angles = {n: v for n, v in zip(L.DOF_NAMES, L.DEFAULT_DOF_POS)}
    _ = Cnfg.control
    _.control_type = 'P'
    _.stiffness = {'joint': 20.}
    _.damping = {'joint': 0.5}
    _.action_scale = 0.25
    _.hip_scale_reduction = 0.5
    _.decimation = 4
    _ = Cnfg.asset
    _.file = '{MINI_GYM_ROOT_DIR}/resources/robots/go1/urdf/go1.urdf'
    _.foot_name = "foot"
    _.penalize_contacts_on = ["thigh", "calf"]
    _.terminate_after_contacts_on = ["base"]
    _.self_collisions = 0
    _.flip_visual_attachments = False
    _.fix_base_link = False
    _ = Cnfg.rewards
    _.soft_dof_pos_limit = 0.9
    _.base_height_target = 0.34
    _ = Cnfg.reward_scales
    _.torques = -0.0001
    _.action_rate = -0.01
    _.dof_pos_limits = -10.0
    _.orientation = -5.
    _.base_height = -30.
    _ = Cnfg.terrain
    _.mesh_type = 'trimesh'
    _.measure_heights = False
    _.terrain_noise_magnitude = 0.0
    _.teleport_robots = True
    _.border_size = 50
    _.terrain_proportions = [0, 0, 0, 0, 0, 0, 0, 0, 1.0]
    _.curriculum = False
    _ = Cnfg.env
    _.num_observations = 42
    _.observe_vel = False
    _.num_envs = 4000
    _ = Cnfg.commands
    _.heading_command = False
    _.resampling_time = 10.0
    _.command_curriculum = True
    _.num_lin_vel_bins = 30
    _.num_ang_vel_bins = 30
    _.lin_vel_x = [-0.6, 0.6]
    _.lin_vel_y = [-0.6, 0.6]
    _.ang_vel_yaw = [-1, 1]
    _ = Cnfg.domain_rand
    _.randomize_base_mass = True
    _.added_mass_range = [-1, 3]
    _.push_robots = False
    _.max_push_vel_xy = 0.5
    _.randomize_friction = True
    _.friction_range = [0.05, 4.5]
    _.randomize_restitution = True
    _.restitution_range = [0.0, 1.0]
    _.restitution = 0.5
    _.randomize_com_displacement = True
    _.com_displacement_range = [-0.1, 0.1]
    _.randomize_motor_strength = True
    _.motor_strength_range = [0.9, 1.1]
    _.randomize_Kp_factor = False
    _.randomize_Kd_factor = False
    _.rand_interval_s = 6


TRAIN_FLAGS = (
    # scripts/train.py:296-338: (flag, argparse kwargs) -- the env / reward flags train_go1 reads
    ("--strategy", dict(default="vel", choices=["e2e", "pms", "vel"])),
    ("--exploration_steps", dict(type=int, default=2500)),
    ("--command_type", dict(default="xy", choices=["xy", "6dof", "xy_norm"])),
    ("--timestep_in_obs", dict(action="store_true")),
    ("--num_history", dict(type=int, default=1)),
    ("--measure_front_half", dict(action="store_true")),
    ("--rotate_camera", dict(action="store_true")),
    ("--camera_zero", dict(action="store_true")),
    ("--blind", dict(action="store_true")),
    ("--terminal_body_height", dict(type=float, default=0.0)),
    ("--terrain", dict(default="single_path", choices=["single_path", "multi_path", "plane"])),
    ("--no_domain_rand", dict(action="store_true")),
    ("--empty_tunnel", dict(action="store_true")),
    ("--random_target", dict(action="store_true")),
    ("--terminate_after_reach", dict(action="store_true")),
    ("--tunnel_width", dict(type=float, default=2.0)),
    ("--lin_vel_form", dict(default="exp", choices=["l1", "l2", "exp", "prod"])),
    ("--r_explore_lin", dict(type=float, default=1.0)),
    ("--r_explore_yaw", dict(type=float, default=0.4)),
    ("--penalty_scaler", dict(type=float, default=1.0)),
    ("--only_positive", dict(action="store_true")),
    ("--r_orientation", dict(type=float, default=0.0)),
    ("--r_base_height", dict(type=float, default=20.0)),
    ("--r_ang_vel", dict(type=float, default=0.001)),
    ("--t_reach", dict(type=int, default=0)),
    ("--r_task", dict(type=float, default=1.0)),
    ("--r_collision", dict(type=float, default=5.0)),
    ("--r_large_vel", dict(type=float, default=0.0)),
)
README_ARGV = ("--terrain", "single_path", "--measure_front_half", "--camera_zero", "--penalty_scaler", "1.0",
               "--strategy", "e2e", "--terminal_body_height", "0.0")


def parse_train_flags(argv=()):
    import argparse
    p = argparse.ArgumentParser(add_help=False)
    for flag, kw in TRAIN_FLAGS:
        p.add_argument(flag, **kw)
    args, _ = p.parse_known_args(list(argv))
    return args


def train_config(argv=(), n_envs=None, rows=None, cols=None):
    """Cfg exactly as scripts/train.py:train_go1 (:46-241) builds it for the command-line flags
    `argv` (same flag names and defaults, train.py:296-338); num_envs / terrain grid overridable
    (train.py:128-130 hard-codes 1024 / 32 / 32).  Attribute assignments keep the reference's
    order: the reward_scales dict order (the reward summation order, :1380-1397) follows it."""
    args = parse_train_flags(argv)
    C = make_cfg()
    config_go1(C)
    C.env.observe_heights = True
    command_type = args.command_type
    C.env.command_type = command_type
    if command_type in ("xy", "xy_norm"):
        C.env.num_observations = 261 if args.measure_front_half else 503
    else:
        C.env.num_observations = 265 if args.measure_front_half else 507
    C.env.num_observations += int(args.timestep_in_obs)
    C.env.num_scalar_observations = C.env.num_observations
    C.env.num_privileged_obs = 2
    C.terrain.measured_points_x = np.linspace(-1, 1, 21)
    C.terrain.measured_points_y = np.linspace(-0.5, 0.5, 11)
    C.env.num_observation_history = args.num_history
    C.env.look_from_back = True
    C.env.viewer_look_at_robot = False
    C.env.terminate_end_of_trajectory = args.terminate_after_reach
    C.env.record_all_envs = False
    C.env.episode_length_s = 20
    C.env.rotate_camera = args.rotate_camera
    C.env.camera_zero = args.camera_zero
    C.env.timestep_in_obs = args.timestep_in_obs
    C.terrain.measure_front_half = args.measure_front_half
    C.asset.penalize_contacts_on = ["thigh", "calf", "base"]
    C.asset.terminate_after_contacts_on = []
    C.rewards.small_vel_threshold = 0.1
    C.rewards.lin_reaching_criterion = 0.3
    C.rewards.ang_reaching_criterion = np.pi / 20.0
    C.rewards.only_positive_rewards = args.only_positive
    C.rewards.use_terminal_body_height = True
    C.rewards.terminal_body_height = args.terminal_body_height
    C.rewards.lin_vel_form = args.lin_vel_form
    C.rewards.exploration_steps = +np.inf
    C.rewards.tracking_sigma_lin = 0.05
    C.rewards.base_height_target = 0.28
    C.rewards.target_lin_vel = 0.25
    p = args.penalty_scaler
    C.reward_scales.dof_acc = -2.5e-7 * p
    C.reward_scales.torques = -1e-5 * p
    C.reward_scales.action_rate = -1e-3 * p
    C.reward_scales.dof_pos_limits = -10.0 * p
    C.reward_scales.collision = -args.r_collision * p
    C.reward_scales.base_height = -args.r_base_height * p
    C.reward_scales.orientation = -args.r_orientation * p
    C.reward_scales.ang_vel_xy = -args.r_ang_vel * p
    C.reward_scales.large_vel = -args.r_large_vel * p
    C.reward_scales.reaching_z = 0.0
    C.reward_scales.reaching_roll = 0.0
    C.reward_scales.reaching_pitch = 0.0
    if args.strategy == "vel":
        C.reward_scales.e2e = 0
        C.rewards.T_reach = args.t_reach
        C.rewards.exploration_steps = 200000
    if args.strategy == "e2e":
        C.reward_scales.e2e = args.r_task
        C.rewards.T_reach = args.t_reach
        C.rewards.exploration_steps = args.exploration_steps
    elif args.strategy == "pms":
        C.reward_scales.reaching_z = 0.0
        C.reward_scales.reaching_roll = 0.0
        C.reward_scales.reaching_pitch = 0.0
    C.reward_scales.exploration_lin = args.r_explore_lin
    C.reward_scales.exploration_yaw = args.r_explore_yaw
    C.env.num_envs = 1024
    C.terrain.num_cols = 32
    C.terrain.num_rows = 32
    if args.terrain == "plane":
        C.terrain.mesh_type = 'plane'
    elif args.terrain == "single_path":
        C.terrain.terrain_type = "single_path"
        C.terrain.terrain_length = 4.0
        C.terrain.terrain_width = 2.0
        C.terrain.terrain_ratio_x = 0.9
        C.terrain.terrain_ratio_y = 0.5
        C.terrain.ceiling_height = 0.8
        C.terrain.start_loc = 0.32
        C.terrain.p_flat = 0.0 if args.empty_tunnel else 0.9
        C.terrain.p_double = 0.6
        C.env.episode_length_s = 10.0
        C.commands.sampling_based_planning = False
    elif args.terrain == "multi_path":
        C.terrain.terrain_type = "multi_path"
        C.terrain.terrain_length = 3.0
        C.terrain.terrain_width = args.tunnel_width
        C.terrain.terrain_ratio_x = 0.9
        C.terrain.terrain_ratio_y = 0.25
        C.terrain.ceiling_height = 0.8
        C.env.episode_length_s = 8.0
        C.terrain.start_loc = 0.4
        C.commands.sampling_based_planning = True
        C.commands.plan_interval = 100
    if args.random_target:
        C.commands.traj_function = "random_target"
        C.commands.traj_length = 10
        C.commands.num_interpolation = 1
        C.commands.sampling_based_planning = False
    else:
        C.commands.traj_function = "fixed_target"
        C.commands.traj_length = 1
        C.commands.num_interpolation = 1
        C.commands.switch_dist = 0.3
        C.commands.base_x = C.terrain.terrain_length * C.terrain.terrain_ratio_x - 1.0
    if args.blind:
        C.env.observe_heights = False
        C.env.measure_front_half = False  # sets Cfg.env, not Cfg.terrain: no effect (train.py:187)
        if command_type in ("xy", "xy_norm"):
            C.env.num_observations = 45 + int(args.timestep_in_obs) - 4
            C.env.num_scalar_observations = 45 + int(args.timestep_in_obs) - 4
        else:
            C.env.num_observations = 45 + int(args.timestep_in_obs) + 2 + 4
            C.env.num_scalar_observations = 45 + int(args.timestep_in_obs) + 2 + 4
    enable_random = not args.no_domain_rand
    C.domain_rand.lag_timesteps = 6
    C.domain_rand.randomize_lag_timesteps = True
    C.control.control_type = "actuator_net"
    C.domain_rand.randomize_rigids_after_start = False
    C.env.priv_observe_motion = False
    C.env.priv_observe_gravity_transformed_motion = False
    C.domain_rand.randomize_friction_indep = False
    C.env.priv_observe_friction_indep = False
    C.domain_rand.randomize_friction = enable_random
    C.env.priv_observe_friction = True
    C.domain_rand.friction_range = [0.1, 3.0]
    C.domain_rand.randomize_restitution = enable_random
    C.env.priv_observe_restitution = True
    C.domain_rand.restitution_range = [0.0, 0.4]
    C.domain_rand.randomize_base_mass = enable_random
    C.env.priv_observe_base_mass = False
    C.domain_rand.added_mass_range = [-1.0, 3.0]
    C.domain_rand.randomize_gravity = enable_random
    C.domain_rand.gravity_range = [-1.0, 1.0]
    C.domain_rand.gravity_rand_interval_s = 8.0
    C.domain_rand.gravity_impulse_duration = 0.99
    C.env.priv_observe_gravity = False
    C.domain_rand.randomize_com_displacement = False
    C.domain_rand.com_displacement_range = [-0.15, 0.15]
    C.env.priv_observe_com_displacement = False
    C.domain_rand.randomize_ground_friction = enable_random
    C.env.priv_observe_ground_friction = False
    C.env.priv_observe_ground_friction_per_foot = False
    C.domain_rand.ground_friction_range = [0.0, 0.0]
    C.domain_rand.randomize_motor_strength = enable_random
    C.domain_rand.motor_strength_range = [0.9, 1.1]
    C.env.priv_observe_motor_strength = False
    C.domain_rand.randomize_motor_offset = enable_random
    C.domain_rand.motor_offset_range = [-0.02, 0.02]
    C.env.priv_observe_motor_offset = False
    C.domain_rand.push_robots = False
    C.domain_rand.randomize_Kp_factor = False
    C.env.priv_observe_Kp_factor = False
    C.domain_rand.randomize_Kd_factor = False
    C.env.priv_observe_Kd_factor = False
    C.env.priv_observe_body_velocity = False
    C.env.priv_observe_body_height = False
    C.env.priv_observe_desired_contact_states = False
    C.env.priv_observe_contact_forces = False
    C.env.priv_observe_foot_displacement = False
    C.env.priv_observe_gravity_transformed_foot_displacement = False
    C.normalization.friction_range = [0, 1]
    C.normalization.ground_friction_range = [0, 1]
    C.normalization.clip_actions = 10.0
    if n_envs is not None:
        C.env.num_envs = n_envs
    if rows is not None:
        C.terrain.num_rows = rows
    if cols is not None:
        C.terrain.num_cols = cols
    return C


def readme_config(n_envs=4096, terrain="single_path", rows=32, cols=32, camera_zero=None, domain_rand=True,
                  extra_argv=()):
    """Cfg as scripts/train.py:46-241 builds it for the README command
    (--terrain single_path --measure_front_half --camera_zero --old_ppo
    --penalty_scaler 1.0 --strategy e2e --terminal_body_height 0.0), with
    num_envs / terrain grid overridable (train.py:128-130 hard-codes 1024/32/32).
    `extra_argv` appends further train.py flags (variants)."""
    if terrain not in ("plane", "single_path"):
        raise ValueError(f"terrain {terrain!r}: only plane and single_path are on this path")
    if camera_zero is None:
        camera_zero = terrain != "plane"  # plane + camera_zero crashes in the reference (:402)
    argv = ["--terrain", terrain, "--measure_front_half", "--penalty_scaler", "1.0", "--strategy", "e2e",
            "--terminal_body_height", "0.0"]
    if camera_zero:
        argv.append("--camera_zero")
    if not domain_rand:
        argv.append("--no_domain_rand")
    return train_config(argv + list(extra_argv), n_envs=n_envs, rows=rows, cols=cols)


# ------------------------------------------------------------------ derived values
def derived(cfg):
    """Values LeggedRobot._parse_cfg computes (legged_robot_trajectory_tracking.py:1860-1878)."""
    dt = cfg.control.decimation * cfg.sim.dt
    out = dict(dt=dt, max_episode_length=float(np.ceil(cfg.env.episode_length_s / dt)),
               rand_interval=int(np.ceil(cfg.domain_rand.rand_interval_s / dt)),
               gravity_rand_interval=int(np.ceil(cfg.domain_rand.gravity_rand_interval_s / dt)))
    out["gravity_rand_duration"] = int(np.ceil(out["gravity_rand_interval"] * cfg.domain_rand.gravity_impulse_duration))
    scales = {}
    for k, v in vars(cfg.reward_scales).items():
        if v != 0:
            scales[k] = v * dt
    out["reward_scales"] = scales
    return out


def soft_dof_limits(soft=0.9):
    """_process_dof_props soft limits (:702-706) computed in f32 like torch."""
    lim = np.zeros((12, 2), np.float32)
    for i in range(12):
        lo, hi = L.JOINT_LIMITS[i % 3]
        lo, hi = np.float32(lo), np.float32(hi)
        m = (lo + hi) / np.float32(2)
        r = hi - lo
        half = np.float32(0.5) * r * np.float32(soft)
        lim[i, 0] = m - half
        lim[i, 1] = m + half
    return lim


def f32(x):
    return float(np.float32(x))


# Native physics constants (no reference counterpart: PhysX is closed).  One 5 ms
# integrator step per sim step (as PhysX's substeps = 1, legged_robot_trajectory_tracking_config.py:
# 355-356): the contacts are linearly implicit (added masses in the articulated inertias), which keeps
# the penalty contact stable at that step (tools/implicit_contact_study.py)
# Self-collision springs are explicit (the two bodies sit in different legs' ABA chains, so no added mass
# couples them): 2000 N/m and 10 N.s/m keep h w = 0.7 and h d / m = 0.5 on a 0.1 kg link at 5 ms.
PHYSICS = dict(contact_stiffness=2.0e4, contact_damping=80.0, friction_damping=60.0,
               limit_stiffness=2000.0, limit_damping=20.0, n_internal=1, self_stiffness=2000.0, self_damping=10.0)


def set_contact_fields(c, cfg, physics):
    """The native contact model's go1_config fields: penalty constants, restitution (the terrain's
    cfg.terrain.restitution, PhysX's bounce threshold cfg.sim.physx.bounce_threshold_velocity) and the
    self-collision springs (asset.self_collisions == 0 enables them, Isaac Gym's bitwise filter convention).

    Restitution is a deliberate deviation from PhysX: PhysX bounces a rigid contact faster than the
    threshold with e times its impact speed; the penalty contact has no impact event, so e = (env + terrain) / 2
    hands back the fraction e of the contact's damping while a point separates faster than the threshold.  The
    rebound / impact ratio of a 2.6 m/s drop is 0.26 / 0.30 / 0.34 at e = 0 / 0.5 / 1
    (tests/test_self_collision.py::test_restitution_drop_apex_is_pinned), not e."""
    for k in ("contact_stiffness", "contact_damping", "friction_damping", "limit_stiffness", "limit_damping"):
        setattr(c, k, float(physics[k]))
    c.terrain_restitution = f32(_get(cfg, "terrain.restitution", 0.0))
    c.bounce_threshold = f32(_get(cfg, "sim.physx.bounce_threshold_velocity", 0.5))
    on = int(_get(cfg, "asset.self_collisions", 0)) == 0
    c.self_stiffness = float(physics["self_stiffness"]) if on else 0.0
    c.self_damping = float(physics["self_damping"]) if on else 0.0


def _get(cfg, path, default=None):
    obj = cfg
    for part in path.split("."):
        if not hasattr(obj, part):
            return default
        obj = getattr(obj, part)
    return obj


# Cfg values the HIP step implements, checked before a handle is built: anything else raises
# NotImplementedError instead of silently training on different rewards / targets / observations.
#   path -> (allowed values, reference line the value selects)
SUPPORTED = {
    "rewards.only_positive_rewards": ((False, True), "legged_robot_trajectory_tracking.py:341-342"),
    "rewards.only_positive_rewards_ji22_style": ((False, True), ":343-344"),
    "rewards.lin_vel_form": (("exp", "l1", "l2", "prod"), "reward_crawling.py:88-104"),
    "rewards.reward_container_name": (("RewardsCrawling", "TrajectoryTrackingRewards"), ":1373-1377"),
    "env.terminate_end_of_trajectory": ((False, True), ":211-213, reward_crawling.py:64-66"),
    "env.use_terminal_body_rotation": ((False, True), ":215-216"),
    "env.rotate_camera": ((False, True), ":1934-1936"),
    "env.timestep_in_obs": ((False, True), ":375-377"),
    "env.observe_heights": ((True, False), ":388-423"),
    # "6dof" fails in the reference itself: commands (n, 6) * commands_scale, while command_xy_only
    # (config.py:70, True) sizes the noise vector for 2 commands (:1109); "xy_norm" normalises by
    # the norm over ALL envs' commands (:803-807), a grid-wide reduction this step does not do
    "env.command_type": (("xy",), ":801-816"),
    "env.observe_command": ((True,), ":367-377"),
    "env.observe_vel": ((False,), ":445-453"),
    "env.observe_only_ang_vel": ((False,), ":455-457"),
    "env.observe_only_lin_vel": ((False,), ":459-461"),
    "env.observe_yaw": ((False,), ":463-468"),
    "env.observe_contact_states": ((False,), ":470-473"),
    "env.observe_two_prev_actions": ((False,), ":425-427"),
    "env.observe_timing_parameter": ((False,), ":429-431"),
    "env.observe_clock_inputs": ((False,), ":433-435"),
    "terrain.measure_front_half": ((True, False), ":395-399"),
    # with OMPL installed the reference redraws a sub-terrain until a planner finds a path through it
    "terrain.valid_tunnel_only": ((False,), "go1_gym/utils/tunnel.py:101-118 (OMPL validity check)"),
    "commands.traj_function": (("fixed_target", "random_target", "random_goal"), "trajectory_function.py:14-93"),
    "commands.traj_length": (tuple(range(1, 17)), "trajectory_function.py:14-93 (<= GO1_MAX_TRAJ)"),
    "commands.sampling_based_planning": ((False,), ":850-921 (OMPL planner)"),
    "commands.switch_upon_reach": ((True,), ":836-839"),
    "control.control_type": (("actuator_net",), ":957-996"),
    "domain_rand.lag_timesteps": ((6,), ":973-974"),
    "domain_rand.randomize_lag_timesteps": ((True,), ":973-974"),
    "domain_rand.randomize_com_displacement": ((False,), ":735-742"),
    "domain_rand.push_robots": ((False,), ":1055-1071"),
    "domain_rand.randomize_rigids_after_start": ((False,), ":226-228"),
    "curriculum_thresholds.cl_fix_target": ((False,), ":188-196"),
}

# reward functions of each container (reward_crawling.py:18-123, trajectory_tracking_reward.py:17-171):
# reward_scales name -> go1_term name (abi.TERM_IDS)
_RC = ("torques", "dof_acc", "dof_pos_limits", "collision", "action_rate", "base_height", "ang_vel_xy",
       "orientation", "large_vel", "e2e", "exploration_lin", "exploration_yaw", "reaching_z", "reaching_roll",
       "reaching_pitch")
_TT = ("torques", "dof_vel", "dof_acc", "dof_pos", "collision", "action_rate", "dof_pos_limits", "orientation",
       "task_old", "reach_goal", "reach_goal_t", "reach_goal_T", "task", "exploration", "stalling", "linear_vel",
       "lin_vel_z", "ang_vel_xy", "feet_air_time", "survive", "reaching_z", "reaching_roll", "reaching_pitch",
       "reaching_yaw_abs")
CONTAINERS = {
    "RewardsCrawling": {k: k for k in _RC},
    "TrajectoryTrackingRewards": dict({k: k for k in _TT}, reaching_linear_vel="exploration_lin",
                                      reaching_yaw="exploration_yaw"),
}
# TrajectoryTrackingRewards._reward_reaching_local_goal reads env.replan, which exists only with the
# sampling-based planner (:861); that planner is not on this path
_NOT_ON_PATH = {"reaching_local_goal": ":861 (needs the OMPL planner's replan flag)"}


def reward_slots(cfg, scales=None):
    """(names, term ids, indefinite-slot mask) of the reward slots in Cfg.reward_scales order
    (nonzero scales, :1380-1397).  A name the container has no function for gets GO1_T_NONE (the
    reference prints a warning, skips it and keeps a zero episode sum, :1390-1395)."""
    scales = derived(cfg)["reward_scales"] if scales is None else scales
    cname = _get(cfg, "rewards.reward_container_name", "RewardsCrawling")
    if cname not in CONTAINERS:
        raise NotImplementedError(f"reward container {cname!r} is not on the accelerated path")
    cont = CONTAINERS[cname]
    form = _get(cfg, "rewards.lin_vel_form", "exp")
    names, ids, indef = [], [], 0
    for name in scales:
        if name == "termination":
            # both containers lack _reward_termination: the reference raises AttributeError (:349-350)
            raise AttributeError(f"'{cname}' object has no attribute '_reward_termination'")
        if name in _NOT_ON_PATH and cname == "TrajectoryTrackingRewards":
            raise NotImplementedError(f"reward term {name!r}: {_NOT_ON_PATH[name]}")
        term = cont.get(name)
        if term is None:
            print(f"Warning: reward _reward_{name} has nonzero coefficient but was not found!")
            ids.append(abi.GO1_T_NONE)
        else:
            if term == "exploration_lin" and form == "prod" and cname != "RewardsCrawling":
                # TrajectoryTrackingRewards._reward_reaching_linear_vel has no "prod" branch: it returns None
                raise TypeError("unsupported operand type(s) for *: 'NoneType' and 'float' "
                                "(trajectory_tracking_reward.py:143-155 has no 'prod' form)")
            if term in ("exploration", "feet_air_time") or (term == "exploration_lin" and form == "prod"):
                indef |= 1 << len(names)
            ids.append(abi.TERM_IDS[term])
        names.append(name)
    if len(names) > abi.GO1_MAX_TERMS:
        raise NotImplementedError(f"{len(names)} nonzero reward scales; the step supports {abi.GO1_MAX_TERMS}")
    return names, ids, indef


def obs_layout(cfg):
    """Observation row of compute_observations (:357-475) for the supported flags:
    gravity 3, commands 2, dof pos 12, dof vel 12, actions 12, [timestep 1], [heights 2 x points]."""
    ts = int(bool(_get(cfg, "env.timestep_in_obs", False)))
    heights = bool(_get(cfg, "env.observe_heights", True))
    rows = GO1_GRID_ROWS_FRONT if _get(cfg, "terrain.measure_front_half", True) else 21
    n_pts = rows * 11
    width = 41 + ts + (2 * n_pts if heights else 0)
    return {"timestep": ts, "heights": heights, "n_points": n_pts, "height_offset": 41 + ts, "width": width}


GO1_GRID_ROWS_FRONT = 10  # x rows 11..20 of the 21-row grid (:395-399)


def traj_draws(cfg):
    """Uniform draws per reset of the trajectory function (trajectory_function.py:14-93)."""
    kind = _get(cfg, "commands.traj_function", "fixed_target")
    if kind == "random_target":
        return 6 * (int(cfg.commands.traj_length) // int(cfg.commands.num_interpolation) + 1)
    if kind == "random_goal":
        return 3
    return 0


def unsupported(cfg):
    """[(path, value, allowed, reference line)] for every Cfg value the HIP step does not implement."""
    bad = []
    for path, (allowed, ref) in SUPPORTED.items():
        v = _get(cfg, path, allowed[0])
        if isinstance(v, (np.bool_, np.integer)):
            v = v.item()
        if v not in allowed:
            bad.append((path, v, allowed, ref))
    mesh, ttype = _get(cfg, "terrain.mesh_type", "trimesh"), _get(cfg, "terrain.terrain_type", "")
    if mesh != "plane" and ttype != "single_path":
        bad.append(("terrain.terrain_type", ttype, ("single_path",), "tunnel_fn.py:99-163"))
    return bad


def check_supported(cfg):
    bad = unsupported(cfg)
    if bad:
        lines = "; ".join(f"Cfg.{p} = {v!r} (implemented: {', '.join(map(repr, a))}; reference {r})"
                          for p, v, a, r in bad)
        raise NotImplementedError("not on the accelerated path: " + lines)


def build_abi_config(cfg, n_envs=None, physics=None, actuator=None, hf_shape=(80, 40)):
    """go1_config for the C ABI from a (mutated) Cfg (raises NotImplementedError for any Cfg value
    the HIP step does not implement, see SUPPORTED)."""
    check_supported(cfg)
    physics = dict(PHYSICS, **(physics or {}))
    d = derived(cfg)
    c = abi.Go1Config()
    n = n_envs if n_envs is not None else cfg.env.num_envs
    plane = cfg.terrain.mesh_type == "plane"
    c.n_envs = n
    c.terrain_kind = 0 if plane else 1
    c.camera_zero = int(bool(cfg.env.camera_zero))
    if plane and cfg.env.camera_zero:
        raise AttributeError("'LeggedRobot' object has no attribute 'camera_pitch_angle' "
                             "(plane terrain + camera_zero fails in the reference, :402)")
    c.measure_front_half = int(bool(cfg.terrain.measure_front_half))
    ol = obs_layout(cfg)
    if int(cfg.env.num_observations) != ol["width"]:
        # compute_observations asserts the width (:475)
        raise AssertionError(f"Observation shape ({n}, {ol['width']}) does not match num_observations "
                             f"{cfg.env.num_observations}")
    c.num_obs = ol["width"]
    c.observe_heights = int(ol["heights"])
    c.timestep_in_obs = ol["timestep"]
    c.rotate_camera = int(bool(_get(cfg, "env.rotate_camera", False)))
    c.terminate_end_of_trajectory = int(bool(_get(cfg, "env.terminate_end_of_trajectory", False)))
    c.use_terminal_body_rotation = int(bool(_get(cfg, "env.use_terminal_body_rotation", False)))
    names, ids, indef = reward_slots(cfg, d["reward_scales"])
    c.n_terms = len(names)
    for k, t in enumerate(ids):
        c.term_ids[k] = t
    for k in range(len(names), abi.GO1_MAX_TERMS):
        c.term_ids[k] = abi.GO1_T_NONE
    c.term_mask = sum(1 << t for t in set(ids) if t != abi.GO1_T_NONE)
    c.indefinite_slots = indef
    c.live_slots = sum(1 << k for k, t in enumerate(ids) if t != abi.GO1_T_NONE)
    rw = cfg.rewards
    c.reward_mode = 1 if rw.only_positive_rewards else (2 if _get(cfg, "rewards.only_positive_rewards_ji22_style",
                                                                   False) else 0)
    c.sigma_rew_neg = f32(_get(cfg, "rewards.sigma_rew_neg", 5))
    c.lin_vel_form = ("exp", "l1", "l2", "prod").index(_get(cfg, "rewards.lin_vel_form", "exp"))
    used = {t for t in ids}
    need_small = (c.lin_vel_form == 3 and abi.TERM_IDS["exploration_lin"] in used) or \
        abi.TERM_IDS["exploration"] in used or abi.TERM_IDS["stalling"] in used
    need_large = abi.TERM_IDS["task"] in used or abi.TERM_IDS["stalling"] in used
    for attr, need in (("small_vel_threshold", need_small), ("large_dist_threshold", need_large)):
        if need and not hasattr(rw, attr):
            raise AttributeError(f"type object 'rewards' has no attribute '{attr}'")
        setattr(c, attr, f32(getattr(rw, attr, 0.0)))
    cm = cfg.commands
    c.traj_kind = ("fixed_target", "random_target", "random_goal").index(cm.traj_function)
    c.traj_length = int(cm.traj_length)
    c.traj_interp = int(getattr(cm, "num_interpolation", 1))
    if c.traj_kind == 1 and c.traj_length % c.traj_interp != 0:
        raise AssertionError("traj_length % num_interpolation != 0 (trajectory_function.py:73)")
    for k in ("x_range", "y_range", "z_range", "roll_range", "pitch_range", "yaw_range", "x_mean", "y_mean"):
        setattr(c, "traj_" + k, f32(getattr(cm, k, 0.0)))
    c.u_per_env = abi.GO1_U_NOISE + c.num_obs + traj_draws(cfg)
    c.add_noise = int(bool(cfg.noise.add_noise))
    c.use_terminal_body_height = int(bool(cfg.rewards.use_terminal_body_height))
    c.custom_origins = 0 if plane else 1
    c.decimation = cfg.control.decimation
    c.n_internal = physics["n_internal"]
    c.rand_interval = d["rand_interval"]
    c.hf_nx, c.hf_ny = hf_shape
    c.sim_dt = f32(cfg.sim.dt)
    c.dt = f32(d["dt"])
    c.action_scale = f32(cfg.control.action_scale)
    c.hip_scale_reduction = f32(cfg.control.hip_scale_reduction)
    c.clip_actions = f32(cfg.normalization.clip_actions)
    c.clip_obs = f32(cfg.normalization.clip_observations)
    c.horizontal_scale = f32(cfg.terrain.horizontal_scale)
    c.max_episode_length = f32(d["max_episode_length"])
    c.terminal_body_height = f32(cfg.rewards.terminal_body_height)
    c.switch_dist = f32(cfg.commands.switch_dist)
    c.base_height_target = f32(cfg.rewards.base_height_target)
    c.tracking_sigma_lin = f32(cfg.rewards.tracking_sigma_lin)
    c.tracking_sigma_ang = f32(cfg.rewards.tracking_sigma_ang)
    c.target_lin_vel = f32(cfg.rewards.target_lin_vel)
    c.target_ang_vel = f32(cfg.rewards.target_ang_vel)
    c.lin_reaching_criterion = f32(cfg.rewards.lin_reaching_criterion)
    c.ang_reaching_criterion = f32(cfg.rewards.ang_reaching_criterion)
    c.t_reach = f32(getattr(cfg.rewards, "T_reach", 0))
    c.ceiling_height = f32(cfg.terrain.ceiling_height)
    c.obs_scale_dof_pos = f32(cfg.obs_scales.dof_pos)
    c.obs_scale_dof_vel = f32(cfg.obs_scales.dof_vel)
    c.obs_scale_heights = f32(cfg.obs_scales.height_measurements)
    # noise_vec (:1110-1117): torch.ones(k) * scale * level (* obs scale), f32 left to right
    lvl = cfg.noise.noise_level
    ns = cfg.noise_scales
    c.noise_gravity = f32(np.float32(np.float32(1.0) * np.float32(ns.gravity)) * np.float32(lvl))
    c.noise_dof_pos = f32(np.float32(np.float32(np.float32(1.0) * np.float32(ns.dof_pos)) * np.float32(lvl))
                          * np.float32(cfg.obs_scales.dof_pos))
    c.noise_dof_vel = f32(np.float32(np.float32(np.float32(1.0) * np.float32(ns.dof_vel)) * np.float32(lvl))
                          * np.float32(cfg.obs_scales.dof_vel))
    c.camera_offset_x = f32(0.12)
    c.camera_offset_norm = f32(np.sqrt(np.float32(0.12) * np.float32(0.12)))
    fr = cfg.normalization.friction_range
    rr = cfg.normalization.restitution_range
    c.priv_friction_scale = f32(2.0 / (fr[1] - fr[0]))
    c.priv_friction_shift = f32((fr[1] + fr[0]) / 2.0)
    c.priv_rest_scale = f32(2.0 / (rr[1] - rr[0]))
    c.priv_rest_shift = f32((rr[1] + rr[0]) / 2.0)
    dr = cfg.domain_rand
    lo, hi = dr.motor_strength_range
    c.strength_range, c.strength_lo = f32(hi - lo), f32(lo)
    lo, hi = dr.motor_offset_range
    c.offset_range, c.offset_lo = f32(hi - lo), f32(lo)
    if not dr.randomize_motor_strength:
        c.strength_range, c.strength_lo = 0.0, 1.0
    if not dr.randomize_motor_offset:
        c.offset_range, c.offset_lo = 0.0, 0.0
    c.reset_dof_range, c.reset_dof_lo = f32(1.5 - 0.5), f32(0.5)
    c.reset_vel_range, c.reset_vel_lo = f32(0.5 - (-0.5)), f32(-0.5)
    t = cfg.terrain
    c.x_init_range2, c.x_init_lo = f32(t.x_init_range - (-t.x_init_range)), f32(-t.x_init_range)
    c.y_init_range2, c.y_init_lo = f32(t.y_init_range - (-t.y_init_range)), f32(-t.y_init_range)
    c.yaw_range2, c.yaw_lo = f32(t.yaw_init_range - (-t.yaw_init_range)), f32(-t.yaw_init_range)
    c.x_init_offset, c.y_init_offset = f32(t.x_init_offset), f32(t.y_init_offset)
    init = list(cfg.init_state.pos) + list(cfg.init_state.rot) + list(cfg.init_state.lin_vel) + \
        list(cfg.init_state.ang_vel)
    for i, v in enumerate(init):
        c.base_init_state[i] = f32(v)
    cm = cfg.commands
    c.traj_base_x, c.traj_base_y, c.traj_base_z = f32(cm.base_x), f32(cm.base_y), f32(cm.base_z)
    c.traj_roll, c.traj_pitch, c.traj_yaw = f32(cm.base_roll), f32(cm.base_pitch), 0.0
    for i, nme in enumerate(L.DOF_NAMES):
        c.default_dof_pos[i] = f32(cfg.init_state.default_joint_angles[nme])
    soft = soft_dof_limits(getattr(cfg.rewards, "soft_dof_pos_limit", 1.0))
    for i in range(12):
        c.dof_pos_limits[2 * i] = float(soft[i, 0])
        c.dof_pos_limits[2 * i + 1] = float(soft[i, 1])
        c.torque_limits[i] = f32(L.TORQUE_LIMIT)
        lo, hi = L.JOINT_LIMITS[i % 3]
        c.hard_limits[2 * i], c.hard_limits[2 * i + 1] = f32(lo), f32(hi)
    for i, v in enumerate(np.asarray(t.measured_points_x, np.float64)):
        c.height_grid_x[i] = f32(v)
    for i, v in enumerate(np.asarray(t.measured_points_y, np.float64)):
        c.height_grid_y[i] = f32(v)
    set_contact_fields(c, cfg, physics)
    for i, v in enumerate(M.model_block()):
        c.model[i] = float(v)
    w = actuator if actuator is not None else load_actuator()
    for i, v in enumerate(w):
        c.actuator[i] = float(v)
    return c


def load_actuator():
    """Flat f32 actuator weights (GO1_ACTUATOR_FLOATS), from data/actuator_go1.npz."""
    import os
    d = np.load(os.path.join(os.path.dirname(__file__), "data", "actuator_go1.npz"))
    flat = np.concatenate([d["w1"].ravel(), d["b1"], d["w2"].ravel(), d["b2"], d["w3"].ravel(), d["b3"]])
    assert flat.shape == (abi.GO1_ACTUATOR_FLOATS,)
    return flat.astype(np.float32)


def reward_scale_vector(scales: dict, names=None):
    """f32 vector of GO1_MAX_TERMS reward scales in slot order (the order of `names`, default the
    order of `scales`: Cfg.reward_scales order), zero-padded."""
    names = list(scales) if names is None else list(names)
    v = np.zeros(abi.GO1_MAX_TERMS, np.float32)
    for k, name in enumerate(names):
        v[k] = np.float32(scales.get(name, 0.0))
    return v


def _fmaf(a, b, c):
    return np.float32(np.float64(a) * np.float64(b) + np.float64(c))


def gravity_state(gravities):
    """_randomize_gravity (:656-660): sim gravity and normalized gravity_vec, f32.
    torch.norm of a 3-vector is sqrt(fma(z, z, fma(y, y, x*x))) on the CPU."""
    g = np.asarray(gravities, np.float32) + np.array([0, 0, -9.8], np.float32)
    s = np.float32(g[0] * g[0])
    s = _fmaf(g[1], g[1], s)
    s = _fmaf(g[2], g[2], s)
    n = np.sqrt(np.float32(s))
    return g.astype(np.float32), (g / n).astype(np.float32)
