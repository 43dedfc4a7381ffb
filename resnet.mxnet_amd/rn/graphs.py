"""ResNet / ResNeXt graph builders on the mx.sym surface, for runs where the reference tree
is not present (bench.py and the GPU tests run on a box without /root/reference).

Each builder produces the same graph -- node names, parameter names/order, attributes -- as
the reference function it mirrors, so checkpoints and parity fixtures are interchangeable:
  resnet(...)          <-> symbol/resnet.py:77-121   (ResNet-v2, pre-activation bottleneck/basic)
  resnet_cifar10(...)  <-> symbol/resnet.py:123-148  (post-activation basic units)
  resnext(...)         <-> symbol/resnext.py:72-103  (grouped 3x3, BN on the shortcut)
  resnet_int8(...)     <-> symbol/resnet_int8.py:69-131 + int8_api.py:120-171 (fake-quant QAT)
The equivalence is checked against parameter counts and names restated from the reference
(tests/test_symbol_plan.py) -- the reference files themselves are never imported.
"""
import mxnet as mx

BN_EPS = 1e-5


def _bn(x, name, fix_gamma=False, eps=BN_EPS, mom=0.9):
    return mx.sym.BatchNorm(data=x, fix_gamma=fix_gamma, eps=eps, momentum=mom, name=name)


def _relu(x, name):
    return mx.sym.Activation(data=x, act_type="relu", name=name)


def _conv(x, name, nf, k, s=(1, 1), p=(0, 0), g=1, ws=512):
    kw = dict(data=x, num_filter=nf, kernel=k, stride=s, pad=p, no_bias=True, workspace=ws, name=name)
    if g != 1:
        kw["num_group"] = g
    return mx.sym.Convolution(**kw)


def _preact_unit(x, nf, stride, dim_match, name, bottle_neck, mom, ws):
    """Pre-activation unit: returns last_conv + shortcut; the shortcut conv reads act1."""
    a1 = _relu(_bn(x, name + "_bn1", mom=mom), name + "_relu1")
    if bottle_neck:
        specs = [(nf // 4, (1, 1), (1, 1), (0, 0)), (nf // 4, (3, 3), stride, (1, 1)), (nf, (1, 1), (1, 1), (0, 0))]
    else:
        specs = [(nf, (3, 3), stride, (1, 1)), (nf, (3, 3), (1, 1), (1, 1))]
    h = a1
    for i, (f, k, s, p) in enumerate(specs):
        if i > 0:
            h = _relu(_bn(h, "%s_bn%d" % (name, i + 1), mom=mom), "%s_relu%d" % (name, i + 1))
        h = _conv(h, "%s_conv%d" % (name, i + 1), f, k, s, p, ws=ws)
    sc = x if dim_match else mx.sym.Convolution(data=a1, num_filter=nf, kernel=(1, 1), stride=stride, no_bias=True,
                                                workspace=ws, name=name + "_sc")
    return h + sc


def resnet(units, num_stage, filter_list, num_classes, data_type="float32", bottle_neck=True, bn_mom=0.9,
           workspace=512, memonger=False, grad_scale=1.0, dataset_type="imagenet"):
    assert len(units) == num_stage
    data = mx.sym.Variable(name="data")
    data = mx.sym.identity(data=data, name="id") if data_type == "float32" else \
        mx.sym.Cast(data=data, dtype="float16")
    body = _bn(data, "bn_data", fix_gamma=True, eps=2e-5, mom=bn_mom)
    if dataset_type == "imagenet":
        body = _conv(body, "conv0", filter_list[0], (7, 7), (2, 2), (3, 3), ws=workspace)
        body = _relu(_bn(body, "bn0", mom=bn_mom), "relu0")
        body = mx.sym.Pooling(data=body, kernel=(3, 3), stride=(2, 2), pad=(1, 1), pool_type="max")
    elif dataset_type in ("cifar10", "cifar100"):
        body = _conv(body, "conv0", filter_list[0], (3, 3), (1, 1), (1, 1), ws=workspace)
    else:
        raise ValueError("resnet only support imagenet or cifar10 dataset")
    for i in range(num_stage):
        for j in range(units[i]):
            st = (1, 1) if (i == 0 or j > 0) else (2, 2)
            body = _preact_unit(body, filter_list[i + 1], st, j > 0, "stage%d_unit%d" % (i + 1, j + 1), bottle_neck,
                                bn_mom, workspace)
    body = _relu(_bn(body, "bn1", mom=bn_mom), "relu1")
    pool = mx.sym.Pooling(data=body, global_pool=True, kernel=(7, 7), pool_type="avg", name="pool1")
    fc1 = mx.sym.FullyConnected(data=mx.sym.Flatten(data=pool), num_hidden=num_classes, name="fc1")
    if data_type == "float16":
        fc1 = mx.sym.Cast(data=fc1, dtype="float32")
        return mx.sym.SoftmaxOutput(data=fc1, name="softmax", grad_scale=grad_scale)
    return mx.sym.SoftmaxOutput(data=fc1, name="softmax")


def resnet_cifar10(units, num_stage, filter_list, num_classes, data_type="float32", bottle_neck=False, bn_mom=0.9,
                   workspace=512, memonger=False, grad_scale=1.0, dataset_type="cifar10"):
    assert len(units) == num_stage and not bottle_neck
    body = _conv(mx.sym.Variable(name="data"), "conv0", filter_list[0], (3, 3), (1, 1), (1, 1), ws=workspace)
    body = _relu(_bn(body, "bn0", mom=bn_mom), "relu0")
    for i in range(num_stage):
        for j in range(units[i]):
            name = "stage%d_unit%d" % (i + 1, j + 1)
            st = (1, 1) if (i == 0 or j > 0) else (2, 2)
            dim_match = True if j > 0 else filter_list[i] == filter_list[i + 1]
            h = _relu(_bn(_conv(body, name + "_conv1", filter_list[i + 1], (3, 3), st, (1, 1), ws=workspace),
                          name + "_bn1", mom=bn_mom), name + "_relu1")
            h = _bn(_conv(h, name + "_conv2", filter_list[i + 1], (3, 3), (1, 1), (1, 1), ws=workspace),
                    name + "_bn2", mom=bn_mom)
            if dim_match:
                sc = body
            else:
                sc = mx.sym.Convolution(data=body, num_filter=filter_list[i + 1], kernel=(1, 1), stride=st,
                                        no_bias=True, workspace=workspace, name=name + "_sc")
                sc = _bn(sc, name + "_sc_bn", mom=bn_mom)
            body = _relu(h + sc, name + "_relu2")
    pool = mx.sym.Pooling(data=body, global_pool=True, kernel=(7, 7), pool_type="avg", name="pool1")
    fc1 = mx.sym.FullyConnected(data=mx.sym.Flatten(data=pool), num_hidden=num_classes, name="fc1")
    return mx.sym.SoftmaxOutput(data=fc1, name="softmax")


def resnext(units, num_stage, filter_list, num_classes, data_type="float32", num_group=32, bottle_neck=True,
            bn_mom=0.9, workspace=256, memonger=False):
    assert len(units) == num_stage
    width = {32: 0.5, 64: 1.0}[num_group]
    data = mx.sym.Variable(name="data")
    data = mx.sym.identity(data=data, name="id") if data_type == "float32" else \
        mx.sym.Cast(data=data, dtype="float16")
    body = _conv(data, "conv0", filter_list[0], (7, 7), (2, 2), (3, 3), ws=workspace)
    body = _relu(_bn(body, "bn0", mom=bn_mom), "relu0")
    body = mx.sym.Pooling(data=body, kernel=(3, 3), stride=(2, 2), pad=(1, 1), pool_type="max")
    for i in range(num_stage):
        for j in range(units[i]):
            name = "stage%d_unit%d" % (i + 1, j + 1)
            nf = filter_list[i + 1]
            st = (1, 1) if (i == 0 or j > 0) else (2, 2)
            if bottle_neck:
                mid = int(nf * width)
                h = _relu(_bn(_conv(body, name + "_conv1", mid, (1, 1), ws=workspace), name + "_bn1", mom=bn_mom),
                          name + "_relu1")
                h = _relu(_bn(_conv(h, name + "_conv2", mid, (3, 3), st, (1, 1), g=num_group, ws=workspace),
                              name + "_bn2", mom=bn_mom), name + "_relu2")
                h = _bn(_conv(h, name + "_conv3", nf, (1, 1), ws=workspace), name + "_bn3", mom=bn_mom)
            else:
                h = _relu(_bn(_conv(body, name + "_conv1", nf, (3, 3), st, (1, 1), ws=workspace), name + "_bn1",
                              mom=bn_mom), name + "_relu1")
                h = _bn(_conv(h, name + "_conv2", nf, (3, 3), (1, 1), (1, 1), ws=workspace), name + "_bn2",
                        mom=bn_mom)
            if j > 0:
                sc = body
            else:
                sc = _bn(_conv(body, name + "_sc", nf, (1, 1), st, ws=workspace), name + "_sc_bn", mom=bn_mom)
            body = _relu(h + sc, name + "_relu")
    pool = mx.sym.Pooling(data=body, global_pool=True, kernel=(7, 7), pool_type="avg", name="pool1")
    fc1 = mx.sym.FullyConnected(data=mx.sym.Flatten(data=pool), num_hidden=num_classes, name="fc1")
    if data_type == "float16":
        fc1 = mx.sym.Cast(data=fc1, dtype="float32")
    return mx.sym.SoftmaxOutput(data=fc1, name="softmax")


# ----------------------------------------------------------------------------- int8 (QAT) graph
def quant_conv(name, data, num_filter, kernel, stride, pad=(0, 0), no_bias=True, num_group=1, in_channels=None,
               quant_mode="minmax", delay_quant=0, ema_decay=0.99, workspace=512):
    """int8_api.py:120-150 quant_conv_cxx: Quantization_int8 on the weight ('<name>_weight') and on
    the data ('<name>_data') feeding a plain Convolution."""
    weight = mx.sym.Variable(name=name + "_weight", shape=(num_filter, in_channels // num_group) + tuple(kernel),
                             dtype="float32")
    weight_q = mx.sym.contrib.Quantization_int8(data=weight, name=name + "_weight", quant_mode=quant_mode,
                                                is_weight=True, is_weight_perchannel=False, ema_decay=ema_decay,
                                                delay_quant=delay_quant, grad_mode="ste", workspace=workspace)
    data_q = mx.sym.contrib.Quantization_int8(data=data, name=name + "_data", quant_mode=quant_mode, is_weight=False,
                                              is_weight_perchannel=False, ema_decay=ema_decay,
                                              delay_quant=delay_quant, grad_mode="ste", workspace=workspace)
    kw = dict(name=name, data=data_q, num_filter=num_filter, kernel=kernel, stride=stride, pad=pad, no_bias=no_bias,
              weight=weight_q)
    if num_group != 1:
        kw["num_group"] = num_group
    return mx.sym.Convolution(**kw)


def quant_fc(name, data, num_hidden, in_channels, quant_mode="minmax", delay_quant=0, ema_decay=0.99,
             workspace=512):
    """int8_api.py:152-171 quant_fc_cxx."""
    weight = mx.sym.Variable(name=name + "_weight", shape=(num_hidden, in_channels), dtype="float32")
    fc_q = mx.sym.contrib.Quantization_int8(data=weight, name=name + "_weight", is_weight=True, ema_decay=ema_decay,
                                            delay_quant=delay_quant, quant_mode=quant_mode,
                                            is_weight_perchannel=False, grad_mode="ste", workspace=workspace)
    data_q = mx.sym.contrib.Quantization_int8(data=data, name=name + "_data", is_weight=False, ema_decay=ema_decay,
                                              delay_quant=delay_quant, quant_mode=quant_mode,
                                              is_weight_perchannel=False, grad_mode="ste", workspace=workspace)
    return mx.sym.FullyConnected(data=data_q, num_hidden=num_hidden, name=name, weight=fc_q)


def _int8_unit(x, cin, nf, stride, dim_match, name, bottle_neck, mom, qkw):
    """resnet_int8.py:12-66 residual_unit_int8 (pre-activation, every conv quantized)."""
    a1 = _relu(_bn(x, name + "_bn1", mom=mom), name + "_relu1")
    if bottle_neck:
        specs = [(nf // 4, (1, 1), (1, 1), (0, 0)), (nf // 4, (3, 3), stride, (1, 1)), (nf, (1, 1), (1, 1), (0, 0))]
    else:
        specs = [(nf, (3, 3), stride, (1, 1)), (nf, (3, 3), (1, 1), (1, 1))]
    h, c = a1, cin
    for i, (f, k, s, p) in enumerate(specs):
        if i > 0:
            h = _relu(_bn(h, "%s_bn%d" % (name, i + 1), mom=mom), "%s_relu%d" % (name, i + 1))
        h = quant_conv("%s_conv%d" % (name, i + 1), h, f, k, s, p, in_channels=c, **qkw)
        c = f
    sc = x if dim_match else quant_conv(name + "_sc", a1, nf, (1, 1), stride, in_channels=cin, **qkw)
    return h + sc


def resnet_int8(units, num_stage, filter_list, num_classes, data_type="float32", bottle_neck=True, bn_mom=0.9,
                workspace=512, memonger=False, grad_scale=1.0, dataset_type="imagenet", quant_mode="minmax",
                delay_quant=0, ema_decay=0.99):
    """symbol/resnet_int8.py:69-131 (the C5 config graph; BN stays separate)."""
    assert len(units) == num_stage
    qkw = dict(quant_mode=quant_mode, delay_quant=delay_quant, ema_decay=ema_decay, workspace=workspace)
    data = mx.sym.Variable(name="data")
    data = mx.sym.identity(data=data, name="id")
    data = _bn(data, "bn_data", fix_gamma=True, eps=2e-5, mom=bn_mom)
    if dataset_type == "imagenet":
        body = quant_conv("conv0", data, filter_list[0], (7, 7), (2, 2), (3, 3), in_channels=3, **qkw)
        body = _relu(_bn(body, "bn0", mom=bn_mom), "relu0")
        body = mx.sym.Pooling(data=body, kernel=(3, 3), stride=(2, 2), pad=(1, 1), pool_type="max")
    else:
        body = quant_conv("conv0", data, filter_list[0], (3, 3), (1, 1), (1, 1), in_channels=3, **qkw)
    c = filter_list[0]
    for i in range(num_stage):
        st = (1, 1) if i == 0 else (2, 2)
        body = _int8_unit(body, c, filter_list[i + 1], st, False, "stage%d_unit1" % (i + 1), bottle_neck, bn_mom, qkw)
        c = filter_list[i + 1]
        for j in range(units[i] - 1):
            body = _int8_unit(body, c, c, (1, 1), True, "stage%d_unit%d" % (i + 1, j + 2), bottle_neck, bn_mom, qkw)
    body = _relu(_bn(body, "bn1", mom=bn_mom), "relu1")
    pool1 = mx.sym.Pooling(data=body, global_pool=True, kernel=(7, 7), pool_type="avg", name="pool1")
    flat = mx.sym.Flatten(data=pool1)
    fc1 = quant_fc("fc1", flat, num_classes, c, **qkw)
    return mx.sym.SoftmaxOutput(data=fc1, name="softmax")


def resnet50_int8(num_classes=1000):
    return resnet_int8([3, 4, 6, 3], 4, [64, 256, 512, 1024, 2048], num_classes, "float32", True)


def resnet50(num_classes=1000):
    return resnet([3, 4, 6, 3], 4, [64, 256, 512, 1024, 2048], num_classes, "float32", True)


def resnet20_cifar(num_classes=10):
    return resnet_cifar10([3, 3, 3], 3, [16, 16, 32, 64], num_classes, "float32", False, dataset_type="cifar10")


def resnext50_32x4d(num_classes=1000):
    return resnext([3, 4, 6, 3], 4, [64, 256, 512, 1024, 2048], num_classes, "float32", 32, True)
