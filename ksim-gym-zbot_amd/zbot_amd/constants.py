"""Task constants restated from the reference train.py (values, not code)."""

import math

NUM_JOINTS = 20  # train.py:27
NUM_COMMANDS = 6  # train.py:28

# train.py:30-37
ACTOR_DIM = dict(
    joint_positions=20,
    joint_velocity=20,
    imu_orientation=4,
    cmd_linear_velocity=2,
    cmd_absolute_yaw=1,
    cmd_base_height_roll_pitch=3,
)
# train.py:39-51
CRITIC_DIM = dict(
    joint_positions=20,
    joint_velocity=20,
    com_inertia=250,
    com_velocity=150,
    imu_acc=3,
    imu_gyro=3,
    imu_quat=4,
    cmd_all=7,
    act_force=20,
    base_pos=3,
    base_quat=4,
)
NUM_ACTOR_INPUTS = sum(ACTOR_DIM.values())  # 50, train.py:53
NUM_CRITIC_INPUTS = sum(CRITIC_DIM.values())  # 484, train.py:54

COMMAND_NAME = "zero_command"  # train.py:56

# (joint_name, reference_angle_rad, weight) in network-output (= ctrl = qpos[7:]) order, train.py:61-82
JOINT_BIASES: list[tuple[str, float, float]] = [
    ("right_hip_yaw", 0.0, 1.0),
    ("right_hip_roll", -0.1, 1.0),
    ("right_hip_pitch", -0.4, 0.01),
    ("right_knee_pitch", -0.8, 0.01),
    ("right_ankle_pitch", -0.4, 0.01),
    ("right_ankle_roll", -0.1, 0.01),
    ("left_hip_yaw", 0.0, 1.0),
    ("left_hip_roll", 0.1, 1.0),
    ("left_hip_pitch", -0.4, 0.01),
    ("left_knee_pitch", -0.8, 0.01),
    ("left_ankle_pitch", -0.4, 0.01),
    ("left_ankle_roll", 0.1, 0.01),
    ("left_shoulder_pitch", 0.0, 1.0),
    ("left_shoulder_roll", 0.2, 1.0),
    ("left_elbow_roll", -0.2, 1.0),
    ("left_gripper_roll", 0.0, 1.0),
    ("right_shoulder_pitch", 0.0, 1.0),
    ("right_shoulder_roll", -0.2, 1.0),
    ("right_elbow_roll", 0.2, 1.0),
    ("right_gripper_roll", 0.0, 1.0),
]

# Joint groups of the JointDeviationPenalty subclasses (train.py:574-644)
STRAIGHT_LEG_JOINTS = ["left_hip_roll", "left_hip_yaw", "right_hip_roll", "right_hip_yaw"]  # train.py:584-589
ANKLE_KNEE_JOINTS = [  # train.py:605-612
    "left_knee_pitch",
    "left_ankle_pitch",
    "left_ankle_roll",
    "right_knee_pitch",
    "right_ankle_pitch",
    "right_ankle_roll",
]
ARM_POSE_JOINTS = [  # train.py:631-640
    "left_shoulder_pitch",
    "left_shoulder_roll",
    "left_elbow_roll",
    "left_gripper_roll",
    "right_shoulder_pitch",
    "right_shoulder_roll",
    "right_elbow_roll",
    "right_gripper_roll",
]

# Simulation parameters, train.py:1766-1788
NUM_ENVS = 512
ROLLOUT_LENGTH_SECONDS = 4.0
DT = 0.001
CTRL_DT = 0.02
ITERATIONS = 8
LS_ITERATIONS = 8

# Feetech servo deadband, train.py:1111-1118
ENCODER_RESOLUTION = 0.087 * math.pi / 180.0
SERVO_DEADBAND = (2 * ENCODER_RESOLUTION, 2 * ENCODER_RESOLUTION)
VMAX_DEFAULT = 5.0  # train.py:1345
AMAX_DEFAULT = 17.45  # train.py:1346

# Reward registration, train.py:1546-1586: (name, scale, scale_by_curriculum)
REWARDS = [
    ("stay_alive", 1.0, False),
    ("upright", 1.0, False),
    ("naive_forward", 5.0, False),
    ("naive_forward_orientation", 0.3, False),
    ("linear_velocity_penalty_y", -2.0, False),
    ("simple_single_foot_contact", 0.3, False),
    ("feet_airtime", 2.5, False),
    ("feet_orientation", 0.3, False),
    ("feet_too_close", -0.5, False),
    ("straight_leg_penalty", -0.5, True),
    ("ankle_knee_penalty", -0.05, True),
    ("arm_pose_penalty", -2.0, True),
]
