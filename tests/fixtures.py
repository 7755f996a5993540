"""Reference test fixtures and golden outputs.

Inputs are copied (as data) from ``contract/tests/test_contract.cairo``; goldens are the exact
integer outputs listed in SURVEY.md Appendix A.1, themselves reproducing the only hard-coded
expectations of the reference (``test_contract.cairo:285-288``: mu=(20.714, 10.4), rel1 0.533,
rel2 0.647).
"""

# test_contract.cairo:150-158 (constrained, D=2, 7 oracles, f=2)
CONSTRAINED_2D = [
    [492954, 334814], [437692, 410445], [967794, 564219], [431029, 387225],
    [487609, 337990], [284178, 485072], [990059, 558600],
]
# test_contract.cairo:253-261 (unconstrained, max_spread = 10 * WSAD)
UNCONSTRAINED_2D = [
    [20202804, 16401132], [25630344, 13501687], [22210028, 7472938], [18138928, 16619949],
    [19527275, 10116085], [22084988, 7901585], [19549281, 10104796],
]
# test_contract.cairo:355-363 (constrained, D=6)
CONSTRAINED_6D = [
    [444545, 54331, 321181, 93574, 58452, 27915],
    [650669, 423808, 458776, 619552, 867737, 117888],
    [360849, 61583, 445841, 66219, 44810, 20695],
    [442049, 38888, 420748, 44428, 30533, 23350],
    [260736, 619146, 110294, 505377, 699358, 584216],
    [267262, 48987, 551858, 74674, 26617, 30598],
    [268500, 45379, 495298, 145887, 22256, 22678],
]

# name -> (values, constrained, max_spread, golden dict)
GOLDEN = {
    "constrained_2d": (CONSTRAINED_2D, True, 0, dict(
        c1=[462650, 398835],
        qr=[5017, 758, 282522, 1135, 4325, 39289, 303685],
        order=[1, 3, 4, 0, 5, 2, 6],
        reliable=[True, True, False, True, True, True, False],
        consensus=[434360, 362607], rel1=573480, rel2=857846,
        skewness=[-2294596, 1263429], kurtosis=[9083020, 4989576])),
    "unconstrained_2d": (UNCONSTRAINED_2D, False, 10 * 1_000_000, dict(
        c1=[19876042, 10110440],
        qr=[39679579, 44612548, 12403908, 45391272, 121670, 9758482, 106805],
        order=[6, 4, 5, 2, 0, 1, 3],
        reliable=[True, False, True, False, True, True, True],
        consensus=[20714875, 10399307], rel1=533900, rel2=647664,
        skewness=[615187, 2245406], kurtosis=[-391870, 8944662])),
    "constrained_6d": (CONSTRAINED_6D, True, 0, dict(
        c1=[314674, 51659, 433294, 84124, 37671, 25632],
        qr=[29968, 1236241, 2783, 18176, 1356579, 16548, 10077],
        order=[2, 6, 5, 3, 0, 1, 4],
        reliable=[True, False, True, True, False, True, True],
        consensus=[314674, 47183, 433294, 70446, 28575, 23014], rel1=495700, rel2=898314,
        skewness=[-83129, 287925, -671242, 1574887, 1238052, 836244],
        kurtosis=[-187120, 4287271, 5239711, 6998205, 3492635, 2477146])),
}

N_FAILING = 2
ADMINS = [0x416B61736869, 0x4F7A75, 0x48696775636869]      # 'Akashi', 'Ozu', 'Higuchi'
ORACLES = [int.from_bytes(f"oracle_0{i}".encode(), "big") for i in range(7)]
NEW_ORACLE = int.from_bytes(b"oracle_XX", "big")
